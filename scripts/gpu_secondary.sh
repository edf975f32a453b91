#!/bin/bash
# §8(f) kernels: the full -m gpu suite, then scripts/secondary_bench.py (pktgen / to_vec / extract /
# set_fields lines with CPU baselines) and its rocprofv3 kernel stats.
TAG=${1:-r02d}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/gpu_tests.log; grep -E "FAILED|Error" $OUT/gpu_tests.log | head -5
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python scripts/secondary_bench.py > $OUT/secondary.jsonl 2> $OUT/secondary.err
rc=$?; echo "secondary rc=$rc"; cat $OUT/secondary.jsonl; tail -3 $OUT/secondary.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o trace -- \
    python scripts/secondary_bench.py --cpu-budget 0.2 > $OUT/prof_secondary.jsonl 2> $OUT/prof.err
echo "rocprof rc=$?"

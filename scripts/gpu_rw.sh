#!/bin/bash
# Rewrite kernels: flattened to_vec (batched loads) and LDS-window set_fields.  GPU parity, then the
# to_vec / set_fields secondary-bench lines and their rocprof kernel stats.
TAG=${1:-r02za}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -2 $OUT/gpu_tests.log; grep -E "FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit $rc
W=to_vec_c2,to_vec_c4,setfields_c2
timeout -k 10 300 python scripts/secondary_bench.py --only $W > $OUT/secondary.jsonl 2> $OUT/secondary.err || exit $?
cat $OUT/secondary.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o trace -- \
    python scripts/secondary_bench.py --only $W --cpu-budget 0.2 > $OUT/prof_secondary.jsonl 2> $OUT/prof.err || exit $?
grep -h "to_vec\|set_fields\|ipv4_update" $OUT/prof/*kernel_stats.csv

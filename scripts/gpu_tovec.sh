#!/bin/bash
# to_vec rebuilt as one flattened chunk list per wave: GPU parity (to_vec / rewrite / stride tests),
# then the to_vec secondary-bench lines and their rocprof kernel stats.
TAG=${1:-r02z}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -2 $OUT/gpu_tests.log; grep -E "FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/secondary_bench.py --only to_vec_c2,to_vec_c4 > $OUT/secondary.jsonl 2> $OUT/secondary.err || exit $?
cat $OUT/secondary.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o trace -- \
    python scripts/secondary_bench.py --only to_vec_c2,to_vec_c4 --cpu-budget 0.2 > $OUT/prof_secondary.jsonl 2> $OUT/prof.err || exit $?
grep -h "to_vec" $OUT/prof/*kernel_stats.csv

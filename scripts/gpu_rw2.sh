#!/bin/bash
# GPU parity (all), then the secondary lines for extract / set_fields(+checksum) / to_vec with
# rocprof stats.
TAG=${1:-r02rw2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/secondary_bench.py --only extract_c2,setfields_c2,to_vec_c2,to_vec_c4 --cpu-budget 0.5 > $OUT/secondary.jsonl 2> $OUT/secondary.err || exit $?
cut -c1-330 $OUT/secondary.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/secprof -o trace -- \
    python scripts/secondary_bench.py --only extract_c2,setfields_c2 --cpu-budget 0.1 > /dev/null 2> $OUT/secprof.err || exit $?
cut -d, -f1-4 $OUT/secprof/trace_kernel_stats.csv | head -8

#!/bin/bash
# GPU parity on the default build, then to_vec unroll A/B (1 / 4 / 8 chunks in flight per lane),
# interleaved twice, then the secondary lines (all) with rocprof stats.
TAG=${1:-r02tv}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in tv1 tv4 tv8; do
  PKTGPU_LIB=packet-rs_amd/lib/variants/$v.so timeout -k 10 200 python scripts/secondary_bench.py --only to_vec_c2,to_vec_c4 --cpu-budget 0.05 > $OUT/tv_$v.$rep.jsonl 2>/dev/null || exit $?
  python -c "
import json,sys
for l in open('$OUT/tv_$v.$rep.jsonl'): d=json.loads(l); print('$v', d['workload'], d['kernel_us'], 'us', d['roofline']['frac'], d.get('parity_vs_oracle'))"
done; done
timeout -k 10 300 python scripts/secondary_bench.py > $OUT/secondary.jsonl 2> $OUT/secondary.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/secprof -o trace -- \
    python scripts/secondary_bench.py --cpu-budget 0.1 > /dev/null 2> $OUT/secprof.err || exit $?
python -c "
import json
for l in open('$OUT/secondary.jsonl'): d=json.loads(l); print(d['workload'], d['kernel_us'], 'us frac', d['roofline']['frac'], 'parity', d.get('parity_vs_oracle'))"
cut -d, -f1-4 $OUT/secprof/trace_kernel_stats.csv | head -14

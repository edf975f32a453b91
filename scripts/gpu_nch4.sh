#!/bin/bash
# 4-chunk windows for narrow fixed slots in extract / set_fields (default build) vs 5 (base):
# full GPU parity on the default build, then the C2 getter / setter lines interleaved twice.
TAG=${1:-r02nch4}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; tail -1 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in base new; do
  if [ $v = base ]; then export PKTGPU_LIB=$PWD/packet-rs_amd/lib/variants/base.so; else unset PKTGPU_LIB; fi
  timeout -k 10 200 python scripts/secondary_bench.py --only extract_c2,setfields_c2 --cpu-budget 0.05 > $OUT/s_$v.$rep.jsonl 2>/dev/null || exit $?
  python -c "
import json
for l in open('$OUT/s_$v.$rep.jsonl'): d=json.loads(l); print('$v', d['workload'], d['kernel_us'], 'us', d['roofline']['frac'], [v for k,v in d.items() if k.startswith('parity')])"
done; done

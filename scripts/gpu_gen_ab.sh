#!/bin/bash
# A/B of the generator kernels (PKTGPU_GEN_MODE 1 = lane per 16-byte piece, 2 = lane per packet),
# then the pktgen tests under the default.
TAG=${1:-r02e}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for m in 1 2 3 1 2 3; do
  PKTGPU_GEN_MODE=$m timeout -k 10 200 python scripts/secondary_bench.py --only pktgen_clone,pktgen_update,pktgen_new,pktgen_values --cpu-budget 0.1 \
      > $OUT/mode$m.jsonl 2> $OUT/mode$m.err || exit $?
  echo "mode $m"; python -c "
import json,sys
for l in open('$OUT/mode$m.jsonl'): d=json.loads(l); print('  ', d['workload'], d['kernel_us'], d['roofline']['frac'], d['parity_vs_oracle'])"
done
timeout -k 10 300 python -u -m pytest tests/test_pktgen.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pktgen_tests.log 2>&1
rc=$?; tail -2 $OUT/pktgen_tests.log; exit $rc

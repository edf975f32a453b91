#!/bin/bash
# pktgen region kernel: odd-piece LDS rows (pad) vs packed rows (base): parity of the default
# build (= pad) on the pktgen tests, then the pktgen lines per build interleaved twice.
TAG=${1:-r02genpad}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_pktgen.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in base dirty; do
  PKTGPU_LIB=packet-rs_amd/lib/variants/$v.so timeout -k 10 200 python scripts/secondary_bench.py --only pktgen_clone,pktgen_update,pktgen_new,pktgen_values --cpu-budget 0.05 > $OUT/g_$v.$rep.jsonl 2>/dev/null || exit $?
  python -c "
import json
for l in open('$OUT/g_$v.$rep.jsonl'): d=json.loads(l); print('$v', d['workload'], d['kernel_us'], 'us', d['roofline']['frac'], d.get('parity_vs_oracle'))"
done; done

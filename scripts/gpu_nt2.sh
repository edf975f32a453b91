#!/bin/bash
# A/B: non-temporal wide stores in pktgen's region kernel and to_vec (nt) vs plain (base).
TAG=${1:-r02nt2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in base nt; do
  PKTGPU_LIB=packet-rs_amd/lib/variants/$v.so timeout -k 10 200 python scripts/secondary_bench.py --only pktgen_update,pktgen_new,pktgen_values,to_vec_c2,to_vec_c4 --cpu-budget 0.05 > $OUT/s_$v.$rep.jsonl 2>/dev/null || exit $?
  python -c "
import json
for l in open('$OUT/s_$v.$rep.jsonl'): d=json.loads(l); print('$v', d['workload'], d['kernel_us'], 'us', d['roofline']['frac'], [v for k,v in d.items() if k.startswith('parity')])"
done; done

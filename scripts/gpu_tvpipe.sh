#!/bin/bash
# to_vec software pipelining by one round (pipe2) vs none (base): to_vec GPU parity on the default
# build (= pipe2), then the to_vec lines per build interleaved twice.
TAG=${1:-r02tvpipe}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "to_vec or c1" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in base pipe2; do
  PKTGPU_LIB=packet-rs_amd/lib/variants/$v.so timeout -k 10 200 python scripts/secondary_bench.py --only to_vec_c2,to_vec_c4 --cpu-budget 0.05 > $OUT/t_$v.$rep.jsonl 2>/dev/null || exit $?
  python -c "
import json
for l in open('$OUT/t_$v.$rep.jsonl'): d=json.loads(l); print('$v', d['workload'], d['kernel_us'], 'us', d['roofline']['frac'], [v for k,v in d.items() if k.startswith('parity')])"
done; done

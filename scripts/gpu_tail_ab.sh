#!/bin/bash
# Register tail A/B (C4 indexed windows): parity of the default build (tail 4) on the indexed/pcap
# tests, then kbench C4 status/chain/all for tail 4 / 0 / 2, interleaved twice.
TAG=${1:-r02v}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "indexed or pcap or mixed or c4 or lockstep or walk" > $OUT/parity.log 2>&1; rc=$?
tail -3 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in libpktgpu libpktgpu_t0 libpktgpu_t2; do
  PKTGPU_LIB=packet-rs_amd/lib/$v.so timeout -k 10 200 python scripts/kbench.py --config c4 --variants "status;chain;all" --windows 0 --streams 1,2 --rounds 2 --iters 16 > $OUT/$v.$rep.txt 2>&1 || exit $?
  echo "== $v rep $rep"; grep "^w=" $OUT/$v.$rep.txt
done
done

#!/bin/bash
# Cooperative window loads for fixed-stride batches (C2/C3): full GPU parity of the default build,
# then kbench C2 and C3 at their bench columns, coop vs per-lane loads, interleaved twice.
TAG=${1:-r02x}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in libpktgpu libpktgpu_nocoopf; do
  PKTGPU_LIB=packet-rs_amd/lib/$v.so timeout -k 10 200 python scripts/kbench.py --config c2 --variants "status;chain,ether,ipv4,udp" --streams 1,2 --rounds 3 --iters 32 > $OUT/$v.c2.$rep.txt 2>&1 || exit $?
  PKTGPU_LIB=packet-rs_amd/lib/$v.so timeout -k 10 200 python scripts/kbench.py --config c3 --variants "status;chain,ether,vlan,ipv4,tcp,udp" --streams 1,2 --rounds 3 --iters 32 > $OUT/$v.c3.$rep.txt 2>&1 || exit $?
  echo "== $v rep $rep"; grep "streams\]" $OUT/$v.c2.$rep.txt $OUT/$v.c3.$rep.txt
done
done

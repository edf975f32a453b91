#!/bin/bash
# Waves per block 4 (default) / 2 / 1 for C4 (finer dispatch granularity for the launch tail), and C2.
TAG=${1:-r02y}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for v in libpktgpu libpktgpu_wpb2 libpktgpu_wpb1; do
  PKTGPU_LIB=packet-rs_amd/lib/$v.so timeout -k 10 200 python scripts/kbench.py --config c4 --variants "chain;all" --streams 1,2 --rounds 2 --iters 16 > $OUT/$v.c4.$rep.txt 2>&1 || exit $?
  PKTGPU_LIB=packet-rs_amd/lib/$v.so timeout -k 10 200 python scripts/kbench.py --config c2 --variants "chain,ether,ipv4,udp" --streams 1,2 --rounds 3 --iters 32 > $OUT/$v.c2.$rep.txt 2>&1 || exit $?
  echo "== $v rep $rep"; grep -h "streams\]" $OUT/$v.c4.$rep.txt $OUT/$v.c2.$rep.txt
done
done

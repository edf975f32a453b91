#!/bin/bash
# C4 A/B of library builds (same ABI): default, L2 prefetch of the sectors past the window, window
# refill.  Interleaved twice; kbench C4 status/chain/all at the default window and 96 B.
TAG=${1:-r02o}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for v in libpktgpu libpktgpu_nocoop; do
  PKTGPU_LIB=packet-rs_amd/lib/$v.so timeout -k 10 200 python scripts/kbench.py --config c4 --variants "status;chain;all" --windows 0 --streams 1,2 --rounds 2 --iters 16 > $OUT/$v.$rep.txt 2>&1 || exit $?
  echo "== $v rep $rep"; grep "^w=" $OUT/$v.$rep.txt
done
done

#!/bin/bash
# C4 window-width A/B (lockstep walk): 64 B (auto) vs 96 / 128 B per-lane windows, plus a refill build.
TAG=${1:-r02n}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python scripts/kbench.py --config c4 --variants "status;chain;all" --windows 0,96,128 --rounds 3 --iters 16 > $OUT/kbench_c4_windows.txt 2>&1 || exit $?
grep -v amdgpu.ids $OUT/kbench_c4_windows.txt
if [ -f packet-rs_amd/lib/libpktgpu_refill.so ]; then
PKTGPU_LIB=packet-rs_amd/lib/libpktgpu_refill.so timeout -k 10 300 python scripts/kbench.py --config c4 --variants "status;chain;all" --windows 0,96 --rounds 3 --iters 16 > $OUT/kbench_c4_refill.txt 2>&1 || exit $?
grep -v amdgpu.ids $OUT/kbench_c4_refill.txt
fi

#!/bin/bash
# Round 3 build check: full GPU parity suite, C4 timing by window (64 = round-2 width, 0 = auto), request anatomy.
set -u
OUT=gpurun_out/r03b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; tail -5 $OUT/gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/kbench.py --config c4 --variants "status;chain;all" --windows 64,0 --streams 1,2 --rounds 3 --iters 24 > $OUT/kb_c4.txt 2>&1 || exit $?
cat $OUT/kb_c4.txt
WINDOWS="64 0" VARIANTS="status all" bash scripts/gpu_c4anat.sh r03b_anat

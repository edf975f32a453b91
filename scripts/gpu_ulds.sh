#!/bin/bash
# A/B: window reads as unaligned LDS loads (ulds) vs dword pairs + v_alignbyte (base): parity of
# the ulds build on the GPU parse tests, then bench.py C2/C3/C4 interleaved twice.
TAG=${1:-r02ulds}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
PKTGPU_LIB=packet-rs_amd/lib/variants/ulds.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh "c2 c4 c3" "base ulds" 2 > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; exit $rc

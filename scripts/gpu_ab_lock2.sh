#!/bin/bash
# Straight-line lockstep step: all GPU tests, then C4/C3 A/B over waves-per-EU for lockstep kernels.
mkdir -p gpurun_out/r01u
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r01u/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r01u/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh "c4" "base lockwpe6 lockwpe4" 2 2>&1 | tee gpurun_out/r01u/ab.txt

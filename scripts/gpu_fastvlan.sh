#!/bin/bash
# VLAN fast path: all GPU tests, then A/B vs the previous build (base.so) on C3/C2.
mkdir -p gpurun_out/r01w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r01w/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r01w/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh "c3 c2" "base fastvlan" 2 2>&1 | tee gpurun_out/r01w/ab.txt

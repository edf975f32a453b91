#!/bin/bash
# Walk schedule A/B (waterfall = base, sweeps = sweep.so) + parity of the sweep build, and the
# C4 window sweep on the base build.
mkdir -p gpurun_out/r01i
PKTGPU_LIB=packet-rs_amd/lib/variants/sweep.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r01i/parity_sweep.log 2>&1
rc=$?; tail -2 gpurun_out/r01i/parity_sweep.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh "c4 c3 c2" "base sweep" 2 2>&1 | tee gpurun_out/r01i/ab_walk.txt || exit $?
bash scripts/ab_modes.sh 1 "c4:--window 64" "c4:--window 96" "c4:--window 128" "c4:--window 160" "c4:--window 256" 2>&1 | tee gpurun_out/r01i/ab_window.txt

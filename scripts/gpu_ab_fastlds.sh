#!/bin/bash
# FAST_REG=2 (all-fast waves emit from LDS at constant offsets): parity, then A/B vs base / FAST_REG=1.
mkdir -p gpurun_out/r01q
PKTGPU_LIB=packet-rs_amd/lib/variants/fastlds.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r01q/parity.log 2>&1
rc=$?; tail -1 gpurun_out/r01q/parity.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh "c2 c5 c3" "base fastlds fastreg" 2 2>&1 | tee gpurun_out/r01q/ab.txt

#!/bin/bash
# State-agnostic walk (generic.so): full parity suite on it, then A/B vs the waterfall.
mkdir -p gpurun_out/r01r
PKTGPU_LIB=packet-rs_amd/lib/variants/generic.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_hostpath.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r01r/parity.log 2>&1
rc=$?; tail -3 gpurun_out/r01r/parity.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh "c4 c3 c2" "base generic" 2 2>&1 | tee gpurun_out/r01r/ab.txt

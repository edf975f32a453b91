#!/bin/bash
# Same-box A/B: store-shape probe floor; base library (slot fill on) vs FAST_REG=1 vs no slot
# fill, on C2/C3/C4; then the mode parity tests on the base library.
mkdir -p gpurun_out/r01g
timeout -k 10 200 python scripts/probe_store.py > gpurun_out/r01g/probe_store.txt 2>&1 || exit $?
cat gpurun_out/r01g/probe_store.txt
bash scripts/ab_bench.sh "c2 c3 c4" "base fastreg noslotfill" 2 2>&1 | tee gpurun_out/r01g/ab.txt || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r01g/parity.log 2>&1
rc=$?; tail -2 gpurun_out/r01g/parity.log; exit $rc

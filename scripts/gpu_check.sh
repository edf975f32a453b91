#!/bin/bash
# All GPU tests, then the bench on C2/C3/C4 (default knobs).
TAG=${1:-r01s}; mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_modes.sh 1 "c2:" "c3:" "c4:" "c4:--staging 2" 2>&1 | tee gpurun_out/$TAG/bench.txt

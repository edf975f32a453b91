#!/bin/bash
# GPU round (tests, smoke, bench, rocprof, PMC) then the native host-memory path measurement.
TAG=${1:-r01j}
bash scripts/gpu_round.sh $TAG || exit $?
timeout -k 10 300 python scripts/hostpath_native.py --config c2 > gpurun_out/$TAG/hostpath_c2.jsonl 2>&1 || exit $?
timeout -k 10 300 python scripts/hostpath_native.py --config c4 --chunks 131072,262144 > gpurun_out/$TAG/hostpath_c4.jsonl 2>&1
rc=$?; cat gpurun_out/$TAG/hostpath_c2.jsonl gpurun_out/$TAG/hostpath_c4.jsonl; exit $rc

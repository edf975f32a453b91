#!/bin/bash
# Store-shape floor, isolated and 2-stream pipelined, next to bench.py's C2 on the same box.
mkdir -p gpurun_out/r01o
timeout -k 10 200 python scripts/probe_store.py > gpurun_out/r01o/probe.txt 2>&1 || exit $?
bash scripts/ab_modes.sh 2 "c2:" > gpurun_out/r01o/bench.txt 2>&1
rc=$?; cat gpurun_out/r01o/probe.txt gpurun_out/r01o/bench.txt; exit $rc

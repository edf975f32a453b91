#!/bin/bash
# Host-memory path: parity tests, then pinned (zero copy) and pageable (chunked copies) rates.
TAG=${1:-r01l}; mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_hostpath.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/hostpath_tests.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/hostpath_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in c2 c4; do
  timeout -k 10 300 python scripts/hostpath_native.py --config $cfg --chunks 262144 > gpurun_out/$TAG/host_pinned_$cfg.jsonl 2>&1 || exit $?
  timeout -k 10 300 python scripts/hostpath_native.py --config $cfg --pageable --chunks 131072,262144 > gpurun_out/$TAG/host_pageable_$cfg.jsonl 2>&1 || exit $?
done
cat gpurun_out/$TAG/host_*.jsonl | grep path

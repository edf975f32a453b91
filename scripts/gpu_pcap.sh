#!/bin/bash
# Device pcap indexer: parity tests, host-path tests, timing, and a rocprof kernel summary.
TAG=${1:-r01z}; mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_pcap_device.py tests/test_hostpath.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/pcap_tests.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/pcap_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/pcap_index_bench.py > gpurun_out/$TAG/pcap_index.jsonl 2>&1 || { cat gpurun_out/$TAG/pcap_index.jsonl; exit 1; }
cat gpurun_out/$TAG/pcap_index.jsonl
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof_pcap -o pcap -- python scripts/pcap_index_bench.py --reps 10 > gpurun_out/$TAG/pcap_prof.log 2>&1 || { tail -20 gpurun_out/$TAG/pcap_prof.log; exit 1; }
find gpurun_out/$TAG/prof_pcap -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200

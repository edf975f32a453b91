#!/bin/bash
# A/B of pcap-indexer build variants (lib/variants_pcap/*.so) against the product build, interleaved.
TAG=${1:-r01z_ab}; mkdir -p gpurun_out/$TAG
timeout -k 10 200 python -u -m pytest tests/test_pcap_device.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 || { tail -20 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
for r in 1 2; do
  for v in prod packet-rs_amd/lib/variants_pcap/*.so; do
    if [ $v = prod ]; then unset PKTGPU_LIB; else export PKTGPU_LIB=$PWD/$v; fi
    echo -n "$(basename $v) "; timeout -k 10 120 python scripts/pcap_index_bench.py --reps 30 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['device_us'], d['device_min_us'])" || exit 1
  done
done

#!/bin/bash
# pcap indexer region size A/B: parity (tests/test_pcap_device.py) under each build, then the
# blocking-call time interleaved twice, then rocprof kernel stats per build.
TAG=${1:-r02pcapreg}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for v in prod packet-rs_amd/lib/variants_pcap/*.so; do
  if [ $v = prod ]; then unset PKTGPU_LIB; else export PKTGPU_LIB=$PWD/$v; fi
  timeout -k 10 200 python -u -m pytest tests/test_pcap_device.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests_$(basename $v).log 2>&1
  rc=$?; echo "$(basename $v) tests: $(tail -1 $OUT/tests_$(basename $v).log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in prod packet-rs_amd/lib/variants_pcap/*.so; do
    if [ $v = prod ]; then unset PKTGPU_LIB; else export PKTGPU_LIB=$PWD/$v; fi
    echo -n "$(basename $v) "; timeout -k 10 120 python scripts/pcap_index_bench.py --reps 30 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['device_us'], d['device_min_us'])" || exit 1
  done
done
for v in prod packet-rs_amd/lib/variants_pcap/*.so; do
  if [ $v = prod ]; then unset PKTGPU_LIB; else export PKTGPU_LIB=$PWD/$v; fi
  b=$(basename $v .so)
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$b -o trace -- python scripts/pcap_index_bench.py --reps 20 > /dev/null 2>&1 || exit $?
  echo "== $b"; grep pcap_ $OUT/prof_$b/trace_kernel_stats.csv | cut -d, -f1-4
done

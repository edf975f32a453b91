#!/bin/bash
# rocprofv3 kernel stats of every packet-rs_amd/lib/variants/*.so through scripts/pcap_index_bench.py
# (timing only: --no-check).  usage: scripts/pcap_variants.sh TAG
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for v in packet-rs_amd/lib/variants/*.so; do
  n=$(basename $v .so)
  PKTGPU_LIB=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o trace -- \
      python scripts/pcap_index_bench.py --reps 10 --no-check > $OUT/$n.log 2>&1 || { echo "$n failed $?"; exit 1; }
  python - $OUT/$n/trace_kernel_stats.csv $n <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'pcap' in r['Name']: print(sys.argv[2], r['Name'].split('(')[0].split('::')[-1], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
done

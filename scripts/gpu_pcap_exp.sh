#!/bin/bash
# Guess-kernel timing experiments: product vs no-walk vs stage-only (rocprof kernel stats).
TAG=${1:-r01z_exp}; mkdir -p gpurun_out/$TAG; cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in prod packet-rs_amd/lib/variants_pcap/exp1.so packet-rs_amd/lib/variants_pcap/exp2.so; do
  n=$(basename $v .so)
  if [ $v = prod ]; then unset PKTGPU_LIB; else export PKTGPU_LIB=$PWD/$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/$n -o p -- python scripts/pcap_index_bench.py --reps 10 --no-check > gpurun_out/$TAG/$n.log 2>&1 || { tail -5 gpurun_out/$TAG/$n.log; exit 1; }
  find gpurun_out/$TAG/$n -name "*kernel_trace.csv" -delete
  echo "== $n"; find gpurun_out/$TAG/$n -name "p_kernel_stats.csv" -exec python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])): print(r['Name'][:60].split('(')[2] if r['Name'].count('(')>1 else r['Name'][:40], r['Calls'], r['AverageNs'])" {} \;
done

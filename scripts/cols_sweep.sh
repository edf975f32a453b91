#!/bin/bash
# Isolated-launch and pipelined time of parse_kernel per requested column set (bench.py phases).
# usage: scripts/cols_sweep.sh c2 "status;chain;chain,ether,ipv4,udp"
C=${1:-c2}; SETS=${2:-"status;chain;chain,ether,ipv4,udp"}
IFS=';' read -ra A <<< "$SETS"
for cols in "${A[@]}"; do
  timeout -k 10 180 python bench.py --config $C --columns "$cols" --no-cpu-baseline --steps 100 --warmup 20 2>/dev/null |
    python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; g=d['GB/s']['algorithmic_bytes_per_pkt']; print(f\"$C [$cols] B/pkt={g['read']:.0f}+{g['written']:.0f} kernel={r['avg_kernel_us']:.2f}us pipelined={r['pipelined']['device_ms_per_step']*1e3:.2f}us\")" || exit 1
done

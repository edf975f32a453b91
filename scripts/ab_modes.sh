#!/bin/bash
# A/B of launch modes through bench.py itself (same process layout as the driver's bench):
# isolated-launch time (roofline phase) and pipelined per-step device time.
# usage: scripts/ab_modes.sh ROUNDS "c2:--grid -1" "c2:--grid 2" "c4:--staging 2" ...
R=${1:-2}; shift
for r in $(seq 1 $R); do
  for v in "$@"; do
    c=${v%%:*}; flags=${v#*:}
    timeout -k 10 180 python bench.py --config $c --no-cpu-baseline --steps 100 --warmup 20 $flags 2>/dev/null |
      python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(f\"$c [$flags] value={d['value']:.2f} Gpkt/s kernel={r['avg_kernel_us']:.2f}us frac={r['frac']:.3f} pipelined={r['pipelined']['device_ms_per_step']*1e3:.2f}us frac={r['pipelined']['frac']:.3f}\", flush=True)" || exit 1
  done
done

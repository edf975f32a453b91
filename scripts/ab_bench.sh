#!/bin/bash
# A/B library variants (packet-rs_amd/lib/variants/<name>.so) and PKTGPU_* env knobs through
# bench.py itself: isolated-launch time (roofline phase) and pipelined per-step device time.
# usage: scripts/ab_bench.sh "c2 c3" "base tiles:PKTGPU_TILES=1 tiles:PKTGPU_TILES=2" ROUNDS
CFGS=${1:-c2}; VARS=${2:-base}; R=${3:-2}
for r in $(seq 1 $R); do
  for c in $CFGS; do
    for v in $VARS; do
      lib=${v%%:*}; envs=""; [[ "$v" == *:* ]] && envs=${v#*:}
      env PKTGPU_LIB=packet-rs_amd/lib/variants/$lib.so ${envs//,/ } timeout -k 10 180 \
        python bench.py --config $c --no-cpu-baseline --steps 100 --warmup 20 2>/dev/null |
        python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(f\"$c $v value={d['value']:.2f} Gpkt/s kernel={r['avg_kernel_us']:.2f}us frac={r['frac']:.3f} pipelined={r['pipelined']['device_ms_per_step']*1e3:.2f}us frac={r['pipelined']['frac']:.3f}\")" || exit 1
    done
  done
done

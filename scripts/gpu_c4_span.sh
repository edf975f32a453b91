#!/bin/bash
# C4 A/B: default staging (per-lane windows) vs wave-span staging (pkt_ctx_set_staging 2), both
# with the lockstep walk (auto for indexed batches); interleaved, 2 rounds.
TAG=${1:-r01zb}; mkdir -p gpurun_out/$TAG
for r in 1 2; do
  for st in 0 2; do
    f=gpurun_out/$TAG/c4_st${st}_$r.json
    timeout -k 10 200 python bench.py --config c4 --staging $st --steps 100 --warmup 10 > $f 2>/dev/null || exit 1
    python3 - "$f" "$st" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("staging", sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["avg_kernel_us"],
      d["roofline"]["pipelined"]["device_ms_per_step"])
PY
  done
done

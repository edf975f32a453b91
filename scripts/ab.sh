#!/bin/bash
# A/B the library variants in packet-rs_amd/lib/variants/ on one device, interleaved rounds.
# usage: scripts/ab.sh "c2 c3" "status;chain;all" ROUNDS
CFGS=${1:-c2}; VARS=${2:-status;chain}; R=${3:-2}
for r in $(seq 1 $R); do
  for v in packet-rs_amd/lib/variants/*.so; do
    for c in $CFGS; do
      PKTGPU_LIB=$v timeout -k 10 120 python scripts/kbench.py --config $c --streams 1,2 --rounds 3 --variants "$VARS" 2>/dev/null | grep "cols=" | sed "s|^|$(basename $v) $c |"
    done
  done
done

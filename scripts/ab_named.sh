#!/bin/bash
# A/B named library builds on one device, interleaved rounds: "main" = packet-rs_amd/lib/libpktgpu.so,
# any other name = packet-rs_amd/lib/variants/NAME.so (scripts/build_variant.sh).
# usage: scripts/ab_named.sh CFG VARS ROUNDS NAME [NAME ...]
CFG=$1; VARS=$2; R=$3; shift 3
for r in $(seq 1 $R); do
  for name in "$@"; do
    lib=packet-rs_amd/lib/variants/$name.so; [ "$name" = main ] && lib=packet-rs_amd/lib/libpktgpu.so
    PKTGPU_LIB=$lib timeout -k 10 120 python scripts/kbench.py --config $CFG --streams 1,2 --rounds 3 --variants "$VARS" \
      2>&1 | grep "cols=" | sed "s|^|$name $CFG |" || { echo "$name failed"; exit 1; }
  done
done

#!/bin/bash
# SQ instruction/cycle counters of parse_kernel for each library variant (one rocprofv3 --pmc
# pass per variant, kernel-trace only).  usage: scripts/pmc_ab.sh TAG CONFIG COLUMNS "v1 v2 ..."
set -u
TAG=$1; CFG=$2; COLS=$3; VARS=$4
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for v in $VARS; do
  PKTGPU_LIB=packet-rs_amd/lib/variants/$v.so timeout -k 10 240 rocprofv3 --kernel-trace \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM \
    --output-format csv -d $OUT/$v -o pmc -- \
    python scripts/kbench.py --config $CFG --variants "$COLS" --rounds 1 --iters 12 > $OUT/$v.log 2>&1 || exit 1
  mkdir -p $OUT/$v/sq1 && cp $(find $OUT/$v -name "*counter_collection.csv" | head -1) $OUT/$v/sq1/pmc_counter_collection.csv
  echo "== $v"; python scripts/pmc_summary.py $OUT/$v
done

#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) over a kbench variant, over
# the device pcap indexer (config "pcap": scripts/pcap_index_bench.py), or over secondary_bench
# workloads (config "secondary", variant = its --only list).
# usage: scripts/pmc.sh TAG "variant" [config] [extra kbench args]
set -u
TAG=$1; VAR=$2; CFG=${3:-c2}; EXTRA=${4:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
if [ "$CFG" = pcap ]; then PROG="scripts/pcap_index_bench.py --reps 5 --no-check"
elif [ "$CFG" = secondary ]; then PROG="scripts/secondary_bench.py --only $VAR --cpu-budget 0.02 --iters 5"
else PROG="scripts/kbench.py --config $CFG --variants $VAR --rounds 1 --iters 12 $EXTRA"; fi
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- \
      python $PROG > $OUT/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU && \
run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE
echo rc=$?

#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) over secondary_bench workloads.
# usage: scripts/pmc_secondary.sh TAG workloads kernel
set -u
TAG=$1; W=$2; K=$3
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- \
      python scripts/secondary_bench.py --only $W --iters 6 --cpu-budget 0.05 > $OUT/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU && \
run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
python scripts/pmc_summary.py $OUT $K > $OUT/summary.txt
rc=$?; cat $OUT/summary.txt; exit $rc

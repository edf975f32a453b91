#!/bin/bash
# SQ counters of the pcap indexer kernels (two passes over scripts/pcap_index_bench.py).
TAG=${1:-r02pmcpcap}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
  --output-format csv -d $OUT/sq1 -o pmc -- python scripts/pcap_index_bench.py --reps 5 > /dev/null 2> $OUT/sq1.err || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace \
  --pmc SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_BRANCH \
  --output-format csv -d $OUT/sq2 -o pmc -- python scripts/pcap_index_bench.py --reps 5 > /dev/null 2> $OUT/sq2.err || exit $?
for k in pcap_guess_kernel pcap_scan_kernel; do
  echo "== $k"
  mkdir -p $OUT/$k/sq1 $OUT/$k/sq2
  cp $(find $OUT/sq1 -name "*counter_collection.csv" | head -1) $OUT/$k/sq1/pmc_counter_collection.csv
  cp $(find $OUT/sq2 -name "*counter_collection.csv" | head -1) $OUT/$k/sq2/pmc_counter_collection.csv
  python scripts/pmc_summary.py $OUT/$k $k
done

#!/bin/bash
# C4 evidence for the kernel redesign: kbench (status / chain / all columns, windows vs spans),
# PMC of the default C4 launch, and the FETCH_SIZE calibration of scattered per-lane reads.
TAG=${1:-r02c}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python scripts/kbench.py --config c4 --variants "status;chain;all" --rounds 3 --iters 16 > $OUT/kbench_c4.txt 2>&1 || exit $?
timeout -k 10 240 python scripts/kbench.py --config c4 --variants "chain;all" --staging 2 --rounds 3 --iters 16 > $OUT/kbench_c4_span.txt 2>&1 || exit $?
timeout -k 10 240 python scripts/kbench.py --config c3 --variants "chain;chain,ether,vlan,ipv4,tcp,udp" --rounds 3 --iters 16 > $OUT/kbench_c3.txt 2>&1 || exit $?
bash scripts/pmc.sh $TAG/pmc_c4 "all" c4 > $OUT/pmc_c4.log 2>&1 || exit $?
python scripts/pmc_summary.py $OUT/pmc_c4 > $OUT/pmc_c4_summary.txt
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/calib -o pmc -- \
    python scripts/fetch_calib.py $OUT/calib_plan.json > $OUT/calib.log 2>&1 || exit $?
python scripts/fetch_calib_summary.py $OUT/calib $OUT/calib_plan.json $OUT/calib.json
cat $OUT/kbench_c4.txt $OUT/kbench_c4_span.txt $OUT/kbench_c3.txt $OUT/pmc_c4_summary.txt

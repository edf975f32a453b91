#!/bin/bash
# Which L2 memory-side request counters gfx950 exposes, then the calibration probe under
# TCC_EA0_RDREQ / TCC_EA0_RDREQ_32B / TCC_BUBBLE (128-B requests) to derive exact read bytes.
TAG=${1:-r02req}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1
grep -o 'TCC_[A-Z0-9_]*' $OUT/avail.txt | sort -u > $OUT/tcc_counters.txt
wc -l $OUT/tcc_counters.txt; grep -E 'EA0_RD|BUBBLE|RDREQ' $OUT/tcc_counters.txt | tr '\n' ' '; echo
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --output-format csv -d $OUT/calib_req -o pmc -- \
    python scripts/fetch_calib.py $OUT/calib_plan.json > $OUT/calib_req.log 2>&1
echo "calib rc=$?"

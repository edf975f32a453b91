#!/bin/bash
# C4 line requests per launch by column set (status / chain / all): what the reads cost beyond
# the windows.
TAG=${1:-r02c4req}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
for v in status chain all; do
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/pmc_$v -o pmc -- \
    python scripts/kbench.py --config c4 --variants $v --windows 0 --streams 1 --rounds 1 --iters 8 > $OUT/kb_$v.txt 2>&1 || exit $?
python scripts/traffic_req.py $OUT/pmc_$v parse_kernel $OUT/req_$v.json "$TAG c4 $v" | cut -c1-200 || exit $?
done
for v in status all; do
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pmcw_$v -o pmc -- \
    python scripts/kbench.py --config c4 --variants $v --windows 0 --streams 1 --rounds 1 --iters 8 > /dev/null 2>&1 || exit $?
done

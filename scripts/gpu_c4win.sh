#!/bin/bash
# C4 window width under fully cooperative window loads: kbench at 64 (auto) / 112 / 128 B, and the
# request-size PMC pass per width (all columns).
TAG=${1:-r02win}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
timeout -k 10 240 python scripts/kbench.py --config c4 --variants "status;all" --windows 0,112,128 --streams 1,2 --rounds 3 --iters 16 > $OUT/kb.$rep.txt 2>&1 || exit $?
cat $OUT/kb.$rep.txt
done
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
for w in 0 112 128; do
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/pmc_w$w -o pmc -- \
    python scripts/kbench.py --config c4 --variants all --windows $w --streams 1 --rounds 1 --iters 8 > /dev/null 2>&1 || exit $?
python scripts/traffic_req.py $OUT/pmc_w$w parse_kernel $OUT/req_w$w.json "$TAG c4 all w=$w" | cut -c1-230 || exit $?
done

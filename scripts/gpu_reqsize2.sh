#!/bin/bash
# Request-size PMC passes: the calibration probe, then C2 / C3 / C4 bench commands (one stream).
TAG=${1:-r02req2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/calib -o pmc -- \
    python scripts/fetch_calib.py $OUT/calib_plan.json > $OUT/calib.log 2>&1 || exit $?
for cfg in c2 c3 c4; do
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/$cfg -o pmc -- \
    python bench.py --config $cfg --steps 20 --warmup 2 --no-cpu-baseline --no-c5 --streams 1 > $OUT/$cfg.json 2>&1 || exit $?
python scripts/traffic_req.py $OUT/$cfg parse_kernel $OUT/traffic_req_$cfg.json "$TAG $cfg" || exit $?
done

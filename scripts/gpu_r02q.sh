#!/bin/bash
# Round evidence after the lean lockstep walk: full round (tests, smoke, C2 bench, rocprof, PMC),
# then the C4 bench line with its rocprof stats and PMC traffic.
TAG=${1:-r02q}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/gpu_round.sh $TAG || exit $?
echo "== C4 bench"
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $OUT/c4_bench.json 2> $OUT/c4_bench.err || exit $?
cat $OUT/c4_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4prof -o trace -- \
    python bench.py --config c4 --steps 50 --warmup 5 --no-cpu-baseline --streams 1 > /dev/null 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/c4pmc_fetch -o pmc -- \
    python bench.py --config c4 --steps 20 --warmup 2 --no-cpu-baseline --streams 1 > /dev/null 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/c4pmc_write -o pmc -- \
    python bench.py --config c4 --steps 20 --warmup 2 --no-cpu-baseline --streams 1 > /dev/null 2>&1 && \
python scripts/traffic.py $OUT/c4pmc_fetch $OUT/c4pmc_write $OUT/traffic_c4.json parse_kernel "$TAG c4"

#!/bin/bash
# Round evidence on the final tree: gpu_r02u.sh (tests, smoke, C2 bench + rocprof + PMC, C4 bench +
# rocprof + PMC, C3 bench), C3 PMC traffic, then the secondary-kernel lines with rocprof stats.
TAG=${1:-r02final}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
bash scripts/gpu_r02u.sh $TAG || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/c3pmc_fetch -o pmc -- \
    python bench.py --config c3 --steps 20 --warmup 2 --no-cpu-baseline --streams 1 > /dev/null 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/c3pmc_write -o pmc -- \
    python bench.py --config c3 --steps 20 --warmup 2 --no-cpu-baseline --streams 1 > /dev/null 2>&1 && \
python scripts/traffic.py $OUT/c3pmc_fetch $OUT/c3pmc_write $OUT/traffic_c3.json parse_kernel "$TAG c3" || exit $?
timeout -k 10 300 python scripts/secondary_bench.py > $OUT/secondary.jsonl 2> $OUT/secondary.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/secprof -o trace -- \
    python scripts/secondary_bench.py --cpu-budget 0.2 > $OUT/prof_secondary.jsonl 2> $OUT/secprof.err || exit $?
echo "== secondary"; cut -c1-160 $OUT/secondary.jsonl

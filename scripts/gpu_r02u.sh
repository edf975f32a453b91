#!/bin/bash
# Round evidence on the final tree: everything gpu_r02q.sh collects, plus the C3 bench line.
TAG=${1:-r02u}
OUT=gpurun_out/$TAG
bash scripts/gpu_r02q.sh $TAG || exit $?
echo "== C3 bench"
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $OUT/c3_bench.json 2> $OUT/c3_bench.err || exit $?
cat $OUT/c3_bench.json

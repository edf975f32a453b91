#!/bin/bash
# Sanity on a rebuilt tree (GPU tests, smoke, C2 bench) + the FETCH_SIZE calibration of per-lane
# scattered reads (scripts/fetch_calib.py under one --pmc FETCH_SIZE pass).
TAG=${1:-r02calib}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json | cut -c1-400
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/calib -o pmc -- \
    python scripts/fetch_calib.py $OUT/calib_plan.json > $OUT/calib.log 2>&1 || exit $?
python scripts/fetch_calib_summary.py $OUT/calib $OUT/calib_plan.json $OUT/calib.json

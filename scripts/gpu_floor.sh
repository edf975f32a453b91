#!/bin/bash
# Bench lines of C2/C3/C4 with the line-granular floor in their roofline objects.
TAG=${1:-r02w}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for c in c2 c3 c4; do
  extra="--no-cpu-baseline"; [ $c = c2 ] && extra=""
  timeout -k 10 300 python bench.py --config $c $extra > $OUT/${c}_bench.json 2> $OUT/${c}_bench.err || exit $?
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], r['value'], json.dumps(r['roofline']['line_floor']))" $OUT/${c}_bench.json $c
done

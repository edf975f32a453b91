#!/bin/bash
# GPU parity (all), then every secondary line with rocprof stats.
TAG=${1:-r02sec}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; tail -1 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/secondary_bench.py > $OUT/secondary.jsonl 2> $OUT/secondary.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/secprof -o trace -- \
    python scripts/secondary_bench.py --cpu-budget 0.1 > /dev/null 2> $OUT/secprof.err || exit $?
python -c "
import json
for l in open('$OUT/secondary.jsonl'): d=json.loads(l); print(d['workload'], d['kernel_us'], 'us frac', d['roofline']['frac'], [v for k,v in d.items() if k.startswith('parity')])"
python -c "
import csv
for r in csv.DictReader(open('$OUT/secprof/trace_kernel_stats.csv')):
    if 'rocclr' not in r['Name'] and 'at::' not in r['Name']: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')"

#!/bin/bash
# Round-3 baseline on a fresh box: C2/C3/C4 bench lines + the C3 SQ stall profile.
set -u
OUT=gpurun_out/r03a; mkdir -p $OUT
export TMPDIR=/tmp
for c in c2 c3 c4; do
  timeout -k 10 240 python bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-c5 > $OUT/$c.json 2> $OUT/$c.err || exit $?
  echo "== $c"; python -c "import json;d=json.load(open('$OUT/$c.json'));r=d['roofline'];print(d['value'],r['avg_kernel_us'],r['frac'],r['pipelined']['frac'],r['line_floor']['kernel_frac_of_floor'])"
done
bash scripts/pmc.sh r03a_c3pmc "chain,ether,vlan,ipv4,tcp,udp" c3 && python scripts/pmc_summary.py gpurun_out/r03a_c3pmc > $OUT/c3_pmc_summary.txt
rc=$?; cat $OUT/c3_pmc_summary.txt; exit $rc

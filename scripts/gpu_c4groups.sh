#!/bin/bash
# New GPU test (fused setters > 32 specs), then C4 line requests per launch by column group
# (chain + one group each) to find where 'all' reads beyond 'chain'.
TAG=${1:-r02grp}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_rewrite.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
for v in chain chain,ether chain,vlan chain,ipv4 chain,ipv6 chain,tcp chain,udp all; do
  n=${v//,/_}
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/pmc_$n -o pmc -- \
    python scripts/kbench.py --config c4 --variants $v --windows 0 --streams 1 --rounds 1 --iters 8 > $OUT/kb_$n.txt 2>&1 || exit $?
  python scripts/traffic_req.py $OUT/pmc_$n parse_kernel $OUT/req_$n.json "$TAG c4 $v" > /dev/null || exit $?
  python -c "import json;d=json.load(open('$OUT/req_$n.json'));print('$v', int(d['requests_per_launch']['TCC_EA0_RDREQ_sum']))"
  grep 'w=0' $OUT/kb_$n.txt | tail -1
done

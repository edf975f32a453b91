#!/bin/bash
# A/B: non-temporal column stores (ntst) vs plain (base) on C4 / C2 (bench.py, interleaved twice),
# and the C4 request-size PMC pass per build.
TAG=${1:-r02ntst}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
PKTGPU_LIB=packet-rs_amd/lib/variants/ntst.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "c4_pcap or c2_full or ref22" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh "c4 c2" "base ntst" 2 > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
for v in base ntst; do
PKTGPU_LIB=packet-rs_amd/lib/variants/$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/pmc_$v -o pmc -- \
    python bench.py --config c4 --steps 20 --warmup 2 --no-cpu-baseline --no-c5 --streams 1 > /dev/null 2>&1 || exit $?
python scripts/traffic_req.py $OUT/pmc_$v parse_kernel $OUT/req_$v.json "$TAG c4 $v" | cut -c1-120 || exit $?
done

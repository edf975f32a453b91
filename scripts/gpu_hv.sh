#!/bin/bash
# A/B: header reads past the window by 16-byte loads (hv) vs one dword load per dword (base):
# GPU parity on the default build (= hv), bench.py C4/C3/C2 isolated + pipelined interleaved twice,
# C4 request-size PMC per build.
TAG=${1:-r02hv}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh "c4 c3 c2" "base hv" 2 > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
for v in base hv; do
PKTGPU_LIB=packet-rs_amd/lib/variants/$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/pmc_$v -o pmc -- \
    python bench.py --config c4 --steps 20 --warmup 2 --no-cpu-baseline --no-c5 --streams 1 > /dev/null 2>&1 || exit $?
python scripts/traffic_req.py $OUT/pmc_$v parse_kernel $OUT/req_c4_$v.json "$TAG c4 $v" | cut -c1-200 || exit $?
done

#!/bin/bash
# C4 kernel iteration: the full -m gpu suite, kbench C4 (windows, spans) and C3, PMC of the C4 launch.
TAG=${1:-r02l}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 240 python scripts/kbench.py --config c4 --variants "status;chain;all" --rounds 3 --iters 16 > $OUT/kbench_c4.txt 2>&1 || exit $?
timeout -k 10 240 python scripts/kbench.py --config c4 --variants "chain;all" --staging 2 --rounds 3 --iters 16 > $OUT/kbench_c4_span.txt 2>&1 || exit $?
timeout -k 10 240 python scripts/kbench.py --config c3 --variants "chain;chain,ether,vlan,ipv4,tcp,udp" --rounds 3 --iters 16 > $OUT/kbench_c3.txt 2>&1 || exit $?
bash scripts/pmc.sh $TAG/pmc_c4 "all" c4 > $OUT/pmc_c4.log 2>&1 || exit $?
python scripts/pmc_summary.py $OUT/pmc_c4 > $OUT/pmc_c4_summary.txt
grep -v amdgpu.ids $OUT/kbench_c4.txt $OUT/kbench_c4_span.txt $OUT/kbench_c3.txt; cat $OUT/pmc_c4_summary.txt

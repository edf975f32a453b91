#!/bin/bash
# SQ/LDS/TCC counters of the C4 parse (per-lane windows, then wave spans) and of C2 for contrast.
bash scripts/pmc.sh r01h_c4 all c4 && python scripts/pmc_summary.py gpurun_out/r01h_c4 > gpurun_out/r01h_c4/summary.txt && \
bash scripts/pmc.sh r01h_c4span all c4 "--staging 2" && python scripts/pmc_summary.py gpurun_out/r01h_c4span > gpurun_out/r01h_c4span/summary.txt && \
bash scripts/pmc.sh r01h_c2 "chain,ether,ipv4,udp" c2 && python scripts/pmc_summary.py gpurun_out/r01h_c2 > gpurun_out/r01h_c2/summary.txt
rc=$?
for d in r01h_c4 r01h_c4span r01h_c2; do echo "== $d"; cat gpurun_out/$d/summary.txt; done
exit $rc

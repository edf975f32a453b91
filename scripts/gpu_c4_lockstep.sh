#!/bin/bash
# C4 with the lockstep walk: PMC counters, and the window sweep.
bash scripts/pmc.sh r01t_c4 all c4 > /dev/null 2>&1 && python scripts/pmc_summary.py gpurun_out/r01t_c4 > gpurun_out/r01t_c4/summary.txt
rc=$?; cat gpurun_out/r01t_c4/summary.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_modes.sh 1 "c4:--window 64" "c4:--window 96" "c4:--window 128" "c4:--window 144" 2>&1 | tee gpurun_out/r01t_c4/window.txt

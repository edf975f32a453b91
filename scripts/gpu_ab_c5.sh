#!/bin/bash
# Steady state (one 2^24-packet launch, C5 on one GPU) vs 2^20-packet launches: base vs FAST_REG=1.
mkdir -p gpurun_out/r01n
bash scripts/ab_bench.sh "c5 c2" "base fastreg" 2 2>&1 | tee gpurun_out/r01n/ab_c5.txt

#!/bin/bash
# Round-2 evidence: the C2 round (tests, smoke, bench with C5 record + ceiling + CPU variants,
# rocprof stats, PMC traffic), the host's core count, and the `bench.py --gpus 2` launcher
# rehearsed with gloo on the box's one GPU (two ranks share it).
TAG=${1:-r02b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
( nproc; python -c 'import os; print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())'; cat /sys/fs/cgroup/cpu.max 2>&1 ) > $OUT/host.txt
bash scripts/gpu_round.sh ${TAG} || exit $?
echo "== launcher rehearsal (2 ranks, gloo, one GPU)"
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu-baseline \
  > $OUT/launch2_gloo.json 2> $OUT/launch2_gloo.err
rc=$?; cat $OUT/launch2_gloo.json; tail -3 $OUT/launch2_gloo.err; exit $rc

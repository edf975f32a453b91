#!/bin/bash
# Round evidence: full round on C2 (tests, smoke, bench, rocprof, PMC), then bench + rocprof + PMC
# on C3 and C4, then the 2-rank rehearsal of the multi-process path (gloo, one GPU).
TAG=${1:-r01x}
bash scripts/gpu_round.sh ${TAG} || exit $?
SKIP_TESTS=1 bash scripts/gpu_round.sh ${TAG}_c3 --config c3 || exit $?
SKIP_TESTS=1 bash scripts/gpu_round.sh ${TAG}_c4 --config c4 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --config c5 --backend gloo --steps 20 --warmup 5 > gpurun_out/$TAG/c5_2rank_gloo.json 2> gpurun_out/$TAG/c5_2rank_gloo.err
rc=$?; cat gpurun_out/$TAG/c5_2rank_gloo.json; tail -3 gpurun_out/$TAG/c5_2rank_gloo.err; exit $rc

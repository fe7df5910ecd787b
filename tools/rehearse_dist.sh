#!/bin/bash
# Two-rank rehearsal of bench.py on a single-GPU box (both ranks on cuda:0, the FTE
# window exchange over gloo because RCCL needs one device per rank).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline --no-fte --scale-frames 0 \
  --exchange gloo --window-frames ${WINDOW_FRAMES:-2000} > gpurun_out/rehearse_dist.log 2>&1
echo "rc=$?"
tail -3 gpurun_out/rehearse_dist.log

#!/bin/bash
# the driver's multi-GPU launch form at world size 1 on the one-GPU box: torch.distributed.run,
# RCCL process group (JANUS_DIST_FORCE=1), barriers, max-over-ranks, result gather
set -o pipefail
mkdir -p gpurun_out/torchrun1
JANUS_DIST_FORCE=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/torchrun1/bench.log 2>&1 || { tail -30 gpurun_out/torchrun1/bench.log; exit 1; }
grep '"metric"' gpurun_out/torchrun1/bench.log | cut -c1-400

#!/bin/bash
# Round 6: the only multi-rank RCCL path one GPU can run -- ranks sharing the device try
# to join one communicator, RCCL refuses it (duplicate GPU), and every rank must leave
# with the error in rank 0's line instead of hanging (non-blocking communicator, abort);
# 2 and 4 ranks.  OLPE_COMM_DEBUG traces the communicator's steps on stderr.
mkdir -p gpurun_out/r06e
tools/gpu_steps.sh \
  "r06e/share_rccl2:240:OLPE_COMM_DEBUG=1 python bench.py --gpus 2 --share-gpu-rccl --walkers 2048 --steps 2 --warmup 1 --no-cpu-baseline --comm-timeout 120" \
  "r06e/share_rccl4:240:OLPE_COMM_DEBUG=1 python bench.py --gpus 4 --share-gpu-rccl --walkers 2048 --steps 2 --warmup 1 --no-cpu-baseline --comm-timeout 120"

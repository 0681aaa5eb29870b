#!/bin/bash
# 2-rank rehearsal on the 1-GPU box (both ranks on device 0, host group + max-over-ranks,
# no RCCL), the launcher the driver uses for N > 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --share-gpu --steps 5 --warmup 1 > gpurun_out/dist2_share.log 2>&1

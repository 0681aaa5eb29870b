#!/bin/bash
# 2-rank rehearsals on the 1-GPU box with the launcher the driver uses for N > 1: both
# ranks on device 0 with the host group + max-over-ranks timing and no RCCL
# (dist2_share.log), then with the RCCL exchange attempted, which RCCL refuses for two
# ranks on one device: the JSON line must still come out, with comm_error
# (dist2_share_rccl.log)
L="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 300 $L --master-port 29517 bench.py --gpus 2 --share-gpu --steps 5 --warmup 1 > gpurun_out/dist2_share.log 2>&1 && \
timeout -k 10 400 $L --master-port 29527 bench.py --gpus 2 --share-gpu-rccl --steps 5 --warmup 1 --comm-timeout 60 > gpurun_out/dist2_share_rccl.log 2>&1
rc=$?
tail -2 gpurun_out/dist2_share.log | cut -c1-400; tail -4 gpurun_out/dist2_share_rccl.log | cut -c1-600
exit $rc

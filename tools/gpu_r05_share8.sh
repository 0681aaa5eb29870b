#!/bin/bash
# Round 5: eight ranks on one GPU through the bench launcher (--share-gpu), each with its
# own SMU clock sampler (eight concurrent amdsmi sessions), before the driver's 8-GPU run.
mkdir -p gpurun_out/r05s8
tools/gpu_steps.sh \
  "r05s8/bench_gpus8_share:300:python bench.py --gpus 8 --share-gpu --walkers 8192 --steps 10 --no-cpu-baseline --no-alt" \
  "r05s8/bench_gpus4_share:300:python bench.py --gpus 4 --share-gpu --walkers 16384 --steps 10 --no-cpu-baseline --no-alt"

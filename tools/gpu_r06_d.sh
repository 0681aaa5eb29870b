#!/bin/bash
# Round 6, end: the bench lines on the final tree -- the default line as the driver runs
# it, configs[1], configs[4], configs[0], the one-rank RCCL exchange for configs[2] and
# configs[4] (verified), and two ranks sharing the GPU.
mkdir -p gpurun_out/r06d
tools/gpu_steps.sh \
  "r06d/bench:400:python bench.py" \
  "r06d/bench_c1:400:python bench.py --config 1" \
  "r06d/bench_c4:400:python bench.py --config 4" \
  "r06d/bench_c0:300:python bench.py --config 0" \
  "r06d/bench_exchange:300:python bench.py --exchange --verify-exchange --no-cpu-baseline --no-alt" \
  "r06d/bench_c4_exchange:300:python bench.py --config 4 --exchange --verify-exchange --no-cpu-baseline --no-alt" \
  "r06d/bench_gpus2_share:300:python bench.py --gpus 2 --share-gpu --no-cpu-baseline"

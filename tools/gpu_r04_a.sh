#!/bin/bash
# Round 4, first GPU session: the GPU tests on the pruned tree (launcher, comm
# allocation, configs[1] at SURVEY 8(d)'s shape), then the bench lines of every config
# at their new defaults and the 2-rank launcher from a plain process.
mkdir -p gpurun_out/r04a
tools/gpu_steps.sh \
  "r04a/gpu_tests:400:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "r04a/bench_c2:200:python bench.py --steps 20 --warmup 5" \
  "r04a/bench_c1:200:python bench.py --config 1" \
  "r04a/bench_c0:200:python bench.py --config 0" \
  "r04a/bench_c4:200:python bench.py --config 4" \
  "r04a/bench_gpus2:200:python bench.py --gpus 2 --share-gpu --walkers 2048 --steps 2 --no-cpu-baseline"

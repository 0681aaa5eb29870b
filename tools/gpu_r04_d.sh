#!/bin/bash
# Round 4, fourth GPU session: the whole-ensemble tests (configs[3] / configs[4] as eight
# shard contexts vs one context), the long reference chains incl. the round-4 "long2"
# fixtures, and configs[3]'s and configs[4]'s whole ensembles benched on one GPU.
mkdir -p gpurun_out/r04d
tools/gpu_steps.sh \
  "r04d/tests:400:python -u -m pytest tests/test_gpu_whole_ensembles.py tests/test_gpu_long_reference.py -x -q -rA --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "r04d/bench_c3_one_gpu:200:python bench.py --walkers 524288 --no-cpu-baseline --no-alt" \
  "r04d/bench_c4_whole_one_gpu:200:python bench.py --config 4 --walkers 131072 --no-cpu-baseline --no-alt"

#!/bin/bash
# Round 4, third GPU session: the launcher tests on the box (two ranks sharing the GPU,
# two ranks refused without --share-gpu by their PCI ids) and an 8-rank rehearsal of
# `bench.py --gpus 8` with every rank on the one GPU (host group, barrier and max-over-
# ranks timing, moments summed over the host group; no RCCL on a shared device).
mkdir -p gpurun_out/r04c
tools/gpu_steps.sh \
  "r04c/bench_gpu_tests:300:python -u -m pytest tests/test_bench_gpu.py -x -q -rA --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "r04c/bench_gpus8_share:300:python bench.py --gpus 8 --share-gpu --walkers 8192 --steps 4 --warmup 2 --no-cpu-baseline --no-alt" \
  "r04c/bench_gpus4_share:300:python bench.py --gpus 4 --share-gpu --walkers 16384 --steps 4 --warmup 2 --no-cpu-baseline --no-alt"

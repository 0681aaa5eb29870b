#!/bin/bash
# Round 4 final bench lines on the committed tree (counts from the r04 session):
# every config at its SURVEY 8(d) default, with the CPU baselines.
mkdir -p gpurun_out/r04f
tools/gpu_steps.sh \
  "r04f/bench:200:python bench.py --steps 20 --warmup 5" \
  "r04f/bench_c1:200:python bench.py --config 1" \
  "r04f/bench_c4:200:python bench.py --config 4" \
  "r04f/bench_c0:200:python bench.py --config 0"

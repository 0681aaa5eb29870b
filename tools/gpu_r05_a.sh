#!/bin/bash
# Round 5, first GPU pass: the GPU suite (moments fault hook, chunked long chains against
# the reference), the default bench line, and the --gpus 2 --share-gpu rehearsal that
# must print per_rank_kernel_ms / host_overhead_frac.
mkdir -p gpurun_out/r05a
tools/gpu_steps.sh \
  "r05a/gpu_tests:600:python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread" \
  "r05a/bench:300:python bench.py" \
  "r05a/bench_gpus2_share:300:python bench.py --gpus 2 --share-gpu --walkers 16384 --steps 10 --no-cpu-baseline --no-alt"

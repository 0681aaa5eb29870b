#!/bin/bash
# Round 5, end: the bench lines with the final defaults (warm-ups of ~0.5 s, the SMU
# clock settled): the default line as the driver runs it, configs[1], configs[4], and the
# GPU bench tests.
mkdir -p gpurun_out/r05f3
tools/gpu_steps.sh \
  "r05f3/bench:400:python bench.py" \
  "r05f3/bench_c1:400:python bench.py --config 1" \
  "r05f3/bench_c4:400:python bench.py --config 4" \
  "r05f3/bench_c0:300:python bench.py --config 0" \
  "r05f3/bench_tests:300:python -u -m pytest tests/test_bench_gpu.py -v -m gpu --timeout 300 --timeout-method thread"

#!/bin/bash
# Round 5, late: the clock probe (olpe_probe.hip) -- the GPU suite with its test, smoke,
# and the default bench line (as the driver runs it) with clock_ghz_live, twice.
mkdir -p gpurun_out/r05c
tools/gpu_steps.sh \
  "r05c/gpu_tests:900:python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread" \
  "r05c/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r05c/bench_1:400:python bench.py" \
  "r05c/bench_2:200:python bench.py --no-cpu-baseline" \
  "r05c/bench_c4:300:python bench.py --config 4 --no-cpu-baseline"

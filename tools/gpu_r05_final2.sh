#!/bin/bash
# Round 5, end: the GPU suite and smoke on the final tree, then the bench lines with the
# SMU clock (default as the driver runs it, configs[1], configs[4], a 2-rank rehearsal).
mkdir -p gpurun_out/r05f2
tools/gpu_steps.sh \
  "r05f2/gpu_tests:900:python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread" \
  "r05f2/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r05f2/bench:400:python bench.py" \
  "r05f2/bench_c1:400:python bench.py --config 1 --no-cpu-baseline" \
  "r05f2/bench_c4:400:python bench.py --config 4 --no-cpu-baseline" \
  "r05f2/bench_gpus2_share:300:python bench.py --gpus 2 --share-gpu --walkers 16384 --steps 10 --no-cpu-baseline --no-alt"

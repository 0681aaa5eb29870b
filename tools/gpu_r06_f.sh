#!/bin/bash
# Round 6, end: the GPU suite and smoke on the final tree.
mkdir -p gpurun_out/r06f
tools/gpu_steps.sh \
  "r06f/gpu_tests:900:python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread" \
  "r06f/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'"

#!/bin/bash
# Round 5, last: the GPU suite and smoke on the final tree.
mkdir -p gpurun_out/r05l
tools/gpu_steps.sh \
  "r05l/gpu_tests:900:python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread" \
  "r05l/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'"

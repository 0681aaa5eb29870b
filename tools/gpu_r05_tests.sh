#!/bin/bash
# Round 5: the GPU suite alone (and smoke), on the current tree.
mkdir -p gpurun_out/r05t
tools/gpu_steps.sh \
  "r05t/gpu_tests:900:python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread" \
  "r05t/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'"

#!/bin/bash
# Round 4: the whole GPU suite on the current tree, then smoke().
mkdir -p gpurun_out/r04e
tools/gpu_steps.sh \
  "r04e/gpu_tests:600:python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "r04e/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'"

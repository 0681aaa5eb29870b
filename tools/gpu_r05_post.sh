#!/bin/bash
# Round 5: the reference-executed ~20,000-iteration posterior tests with their printed
# figures (walker-mean agreement, centroid distance), and the chunked reference chains.
mkdir -p gpurun_out/r05p
tools/gpu_steps.sh \
  "r05p/posterior:600:python -u -m pytest tests/test_gpu_long_reference.py -v -s -m gpu --timeout 300 --timeout-method thread"

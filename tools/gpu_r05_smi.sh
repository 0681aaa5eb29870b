#!/bin/bash
# Round 5, late: the SMU's view of the GFX clock under the sampler's load (amdsmi).
mkdir -p gpurun_out/r05s
tools/gpu_steps.sh "r05s/smi:300:python -u tools/smi_clock_probe.py" \
  "r05s/gpu_chunk_tests:300:python -u -m pytest tests/test_gpu_long_reference.py -v -m gpu -k chunk_handoffs --timeout 300 --timeout-method thread"

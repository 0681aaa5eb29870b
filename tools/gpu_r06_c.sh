#!/bin/bash
# Round 6: the comm tests once more (Sampler defaults), then the roofline session on the
# final sampler (digest 8af3dda15916e475: the hand-off hold hook's argument and branches).
mkdir -p gpurun_out/r06c
tools/gpu_steps.sh \
  "r06c/comm:300:python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k 'rccl or comm_calls'" \
  || exit $?
tools/roofline_session.sh r06 fast exact c1_fast c4_fast

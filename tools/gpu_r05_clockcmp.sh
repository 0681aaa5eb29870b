#!/bin/bash
# Round 5: the SMU's GFX clock (amdsmi) against the sampler's own s_memtime rate
# (diagnostic -DOLPE_DIAG_SPAN library, tools/clock_compare.py), three rounds of 20
# configs[2] launches, then 60 (the event ring holds 64).
mkdir -p gpurun_out/r05cc
tools/gpu_steps.sh \
  "r05cc/cmp20:300:OLPE_LIB=diag/span/libolpe.so python -u tools/clock_compare.py 20 5" \
  "r05cc/cmp60:300:OLPE_LIB=diag/span/libolpe.so python -u tools/clock_compare.py 60 5"

#!/bin/bash
# (ran on a tree with the 16-wave ring restored and this change; both removed after it)
# Round 5: the ring sweep's shape-table rows read from a VGPR base with immediate offsets
# (no per-block SGPR->VGPR address copies).  The 16-wave ring's and the ring tests, then a
# same-box A/B of configs[4]: the committed library (diag/base) against this one at 12
# and 16 waves, alternating, twice.
mkdir -p gpurun_out/r05hv
B="python bench.py --config 4 --no-cpu-baseline --no-alt --no-csv"
tools/gpu_steps.sh \
  "r05hv/tests:600:python -u -m pytest tests -x -v -m gpu -k 'ring or c128' --timeout 300 --timeout-method thread" \
  "r05hv/base_a:200:OLPE_LIB=diag/base/libolpe.so $B" \
  "r05hv/new12_a:200:OLPE_RING=12 $B" \
  "r05hv/new16_a:200:OLPE_RING=16 $B" \
  "r05hv/base_b:200:OLPE_LIB=diag/base/libolpe.so $B" \
  "r05hv/new12_b:200:OLPE_RING=12 $B" \
  "r05hv/new16_b:200:OLPE_RING=16 $B"

#!/bin/bash
# Round 3: the single-slot shape table's stale-set rebuild (product) and the windowed
# ring (diag/win, -DOLPE_RING_WINDOW=1) -- parity first, then same-box A/B against the
# previous product build (diag/prev).
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_steps.sh \
  "win_parity_product:400:python -u -m pytest tests/test_gpu_parity.py -q -m gpu -rf --timeout 120 --timeout-method thread" \
  "win_parity_ring:300:OLPE_LIB=diag/win/libolpe.so python -u -m pytest tests/test_gpu_parity.py -q -m gpu -rf -k 'ring or configs4' --timeout 120 --timeout-method thread" \
  "ab_c4_win:400:AB_ARGS='--config 4' tools/ab_libs.sh prev win" \
  "ab_c2_hc:300:tools/ab_libs.sh prev"

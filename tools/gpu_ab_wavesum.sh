#!/bin/bash
# GPU tests on the product library (MFMA chi^2 wave sum), then A/B against the DPP-tree
# build (diag/dpp, -DOLPE_WAVESUM_DPP) on configs[2] fast / exact, [1] and [4].
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "gpu_tests:300:python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread" \
  "smoke:120:python __graft_entry__.py smoke" \
  "ab_c2:200:tools/ab_libs.sh dpp" \
  "ab_c1:200:AB_ARGS='--config 1 --steps 200 --warmup 50' tools/ab_libs.sh dpp" \
  "ab_c4:200:AB_ARGS='--config 4' tools/ab_libs.sh dpp" \
  "ab_exact:300:AB_ARGS='--mode exact --steps 4' tools/ab_libs.sh dpp"

#!/bin/bash
# One-round FAST launches at 16 waves with progress balancing (the new default for
# W <= 16 x CUs): GPU tests + smoke, then configs[1] and 3,500 walkers against the
# 12-wave sampler (OLPE_WPB=12).
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "gpu_tests:300:python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread" \
  "smoke:120:python __graft_entry__.py smoke" \
  "ab_bal_c1:300:AB_ARGS='--config 1 --steps 200 --warmup 50' tools/ab_env.sh OLPE_WPB=12" \
  "ab_bal_2k:300:AB_ARGS='--walkers 3500 --steps 200 --warmup 50' tools/ab_env.sh OLPE_WPB=12 OLPE_WPB=16"

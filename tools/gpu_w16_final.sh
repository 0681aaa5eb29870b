#!/bin/bash
# The 16-wave default for large 2-source 64x64 FAST launches: GPU tests + smoke, then
# configs[2] / [1] against the 12-wave sampler forced by OLPE_WPB=12 (same library).
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "gpu_tests:300:python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread" \
  "smoke:120:python __graft_entry__.py smoke" \
  "ab_w16d_c2:300:tools/ab_env.sh OLPE_WPB=12" \
  "ab_w16d_c1:300:AB_ARGS='--config 1 --steps 200 --warmup 50' tools/ab_env.sh OLPE_WPB=12"

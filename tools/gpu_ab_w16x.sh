#!/bin/bash
# EXACT at 16 waves (draw tables without the accept thresholds fit 16 slices beside the
# cutout): parity tests with OLPE_WPB=16, then A/B against 12 waves on configs[2] / [1].
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "w16x_tests:200:OLPE_WPB=16 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k 'trajectories_match_reference and (c64-exact or c32-exact) or exact_sampler_chi2_bitwise and 64-2 or long_run_matches'" \
  "ab_w16x_c2:400:AB_ARGS='--mode exact --steps 4' tools/ab_env.sh OLPE_WPB=16" \
  "ab_w16x_c1:300:AB_ARGS='--mode exact --config 1 --steps 40 --warmup 10' tools/ab_env.sh OLPE_WPB=16"

#!/bin/bash
# 16 waves per workgroup for the 2-source 64x64 FAST sampler (single shape-table slot):
# parity tests with OLPE_WPB=16, then A/B on configs[2] / [1] against the 12-wave default:
# the product library at 16 waves (two-row update, no shape-table prefetch) and the
# four-row-update build (diag/w16ru4, -DOLPE_ROWU=4).
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "w16_tests:200:OLPE_WPB=16 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k 'bench_size or long_run_64 or walker_queue or work_units_equal or trajectories'" \
  "w16ru4_tests:200:OLPE_WPB=16 OLPE_LIB=diag/w16ru4/libolpe.so python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k 'bench_size or long_run_64 or walker_queue or work_units_equal or trajectories'" \
  "ab_w16_c2:300:tools/ab_env.sh OLPE_WPB=16 'OLPE_WPB=16 OLPE_LIB=diag/w16ru4/libolpe.so'" \
  "ab_w16_c1:300:AB_ARGS='--config 1 --steps 200 --warmup 50' tools/ab_env.sh OLPE_WPB=16 'OLPE_WPB=16 OLPE_LIB=diag/w16ru4/libolpe.so'"

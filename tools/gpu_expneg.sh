#!/bin/bash
# exp_neg: bit-for-bit check against ocml's exp, GPU tests, EXACT-mode A/B against the
# library of HEAD (diag/head, tools/build_rev.sh HEAD head).
export TMPDIR=/tmp
timeout -k 10 120 tools/micro/exp_check > gpurun_out/exp_check.log 2>&1 && \
tools/gpu_steps.sh "gpu_tests:400:python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread" && \
AB_ARGS="--mode exact --steps 4" timeout -k 10 400 tools/ab_libs.sh head > gpurun_out/ab_expneg.log 2>&1 && \
AB_ARGS="--mode exact --steps 4 --config 4" timeout -k 10 400 tools/ab_libs.sh head > gpurun_out/ab_expneg_c4.log 2>&1

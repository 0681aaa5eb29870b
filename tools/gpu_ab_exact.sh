#!/bin/bash
# GPU tests, then EXACT-mode A/B of the working tree against diag/<base> (tools/build_rev.sh)
#   usage: tools/gpu_ab_exact.sh <base> [tag]
export TMPDIR=/tmp
b=${1:-expneg}; t=${2:-exact}
tools/gpu_steps.sh "gpu_tests:400:python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread" && \
AB_ARGS="--mode exact --steps 4" timeout -k 10 400 tools/ab_libs.sh $b > gpurun_out/ab_${t}.log 2>&1 && \
AB_ARGS="--mode exact --steps 40 --config 1" timeout -k 10 400 tools/ab_libs.sh $b > gpurun_out/ab_${t}_c1.log 2>&1

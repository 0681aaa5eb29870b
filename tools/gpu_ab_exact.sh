#!/bin/bash
# GPU tests, then EXACT-mode A/B of the working tree against diag/<base> (tools/build_rev.sh)
# on configs[2] and configs[1] (and configs[4] with C4=1).
#   usage: [C4=1] tools/gpu_ab_exact.sh <base> [tag]
export TMPDIR=/tmp
b=${1:-expneg}; t=${2:-exact}
tools/gpu_steps.sh "gpu_tests:400:python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread" || exit 1
AB_ARGS="--mode exact --steps 4" timeout -k 10 400 tools/ab_libs.sh $b > gpurun_out/ab_${t}.log 2>&1 || exit 1
AB_ARGS="--mode exact --steps 40 --config 1" timeout -k 10 400 tools/ab_libs.sh $b > gpurun_out/ab_${t}_c1.log 2>&1 || exit 1
if [ -n "$C4" ]; then
  AB_ARGS="--mode exact --steps 3 --config 4" timeout -k 10 400 tools/ab_libs.sh $b > gpurun_out/ab_${t}_c4.log 2>&1 || exit 1
fi

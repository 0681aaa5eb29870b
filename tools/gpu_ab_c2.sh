#!/bin/bash
# GPU tests, then a same-box A/B of the product library against diag/prev (configs[2]
# and configs[1]) and the SQ VALU count of configs[2]: tools/gpu_ab_c2.sh <tag>
export TMPDIR=/tmp
tag=${1:-ab}
tools/gpu_steps.sh \
  "gpu_tests:400:python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread" \
  "ab_c2:300:tools/ab_libs.sh prev" \
  "ab_c1:300:AB_ARGS='--config 1' tools/ab_libs.sh prev" && \
timeout -k 10 200 tools/pmc_valu.sh 2 fast $tag > /dev/null 2>&1; tail -1 gpurun_out/valu_fast.log | cut -c1-120

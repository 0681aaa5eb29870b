#!/bin/bash
# One GPU round trip after a kernel change: GPU tests, smoke, SQ VALU counts of configs[2]
# fast (gpurun_out/pmc_<tag>_valu_fast) and a bench line.  usage: tools/gpu_check.sh <tag>
export TMPDIR=/tmp
tag=${1:-chk}
tools/gpu_steps.sh \
  "gpu_tests:300:python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread" \
  "smoke:120:python __graft_entry__.py smoke" && \
timeout -k 10 200 tools/pmc_valu.sh 2 fast $tag && \
tools/gpu_steps.sh "bench:300:python bench.py --no-cpu-baseline" ${EXTRA_STEPS:+"$EXTRA_STEPS"}

#!/bin/bash
# Round-2 refresh on HEAD: GPU tests + smoke, SQ VALU counts of the current kernel
# (profiles/valu_counts.json, so bench's roofline is not stale), kernel stats, bench.
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "gpu_tests:300:python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread" \
  "smoke:120:python __graft_entry__.py smoke" && \
timeout -k 10 200 tools/pmc_valu.sh 2 fast r02 && \
timeout -k 10 300 tools/pmc_valu.sh 2 exact r02 && \
timeout -k 10 200 tools/pmc_valu.sh 1 fast r02 && \
timeout -k 10 200 tools/pmc_valu.sh 4 fast r02 && \
tools/gpu_steps.sh \
  "prof_fast:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02_fast -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-alt --mode fast" \
  "bench:300:python bench.py"

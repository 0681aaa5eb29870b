#!/bin/bash
# r02 kernel change: parity, bench, SQ VALU counts for every bench config
tools/gpu_steps.sh \
 "gpu_tests:600:python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread" \
 "bench:200:python bench.py --no-cpu-baseline" && \
timeout -k 10 200 tools/pmc_valu.sh 2 fast r02 && timeout -k 10 200 tools/pmc_valu.sh 2 exact r02 && \
timeout -k 10 200 tools/pmc_valu.sh 1 fast r02 && timeout -k 10 200 tools/pmc_valu.sh 4 fast r02

#!/bin/bash
tools/gpu_steps.sh \
 "gpu_tests:600:python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread" && \
timeout -k 10 200 tools/pmc_valu.sh 2 fast r02 && \
timeout -k 10 400 tools/ab_libs.sh prev > gpurun_out/ab_prev.log 2>&1

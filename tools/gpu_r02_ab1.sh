#!/bin/bash
# work-unit A/B: chunks per walker for configs[1] and configs[2]
tools/gpu_steps.sh "units_tests:300:python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k work_units --timeout 120 --timeout-method thread" && \
AB_ARGS="--config 1" timeout -k 10 300 tools/ab_env.sh OLPE_UNITS=1 OLPE_UNITS=2 OLPE_UNITS=3 OLPE_UNITS=4 OLPE_UNITS=6 OLPE_UNITS=8 OLPE_UNITS=12 > gpurun_out/ab_units_c1.log 2>&1 && \
AB_ARGS="--config 2" timeout -k 10 300 tools/ab_env.sh OLPE_UNITS=1 OLPE_UNITS=2 OLPE_UNITS=3 OLPE_UNITS=6 > gpurun_out/ab_units_c2.log 2>&1

#!/bin/bash
tools/gpu_steps.sh \
 "c4_tests:600:python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread -k '128 or configs4 or l2_sampler or other_cutout'" \
 "gpu_tests:600:python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread" \
 "bench_c4:200:python bench.py --config 4 --no-cpu-baseline" \
 "bench_c4_prev:200:OLPE_LIB=diag/prev/libolpe.so python bench.py --config 4 --no-cpu-baseline --no-alt" \
 "bench_c4b:200:python bench.py --config 4 --no-cpu-baseline --no-alt" && \
timeout -k 10 200 tools/pmc_valu.sh 4 fast r02

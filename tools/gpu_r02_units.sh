#!/bin/bash
# r02 work units: GPU tests, benches and kernel stats
tools/gpu_steps.sh \
 "gpu_tests:600:python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread" \
 "bench:200:python bench.py" \
 "bench_c1:200:python bench.py --config 1" \
 "bench_c1_p1:200:OLPE_UNITS=1 python bench.py --config 1 --no-cpu-baseline --no-alt" \
 "bench_c4:200:python bench.py --config 4" \
 "bench_c4_p1:200:OLPE_UNITS=1 python bench.py --config 4 --no-cpu-baseline --no-alt" \
 "prof_c1:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02_c1_fast -o run --output-format csv -- python bench.py --config 1 --no-cpu-baseline --no-alt" \
 "prof_fast:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02_fast -o run --output-format csv -- python bench.py --no-cpu-baseline --no-alt --steps 5 --warmup 1"

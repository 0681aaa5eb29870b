tools/gpu_steps.sh \
 "units_tests:300:python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k work_units --timeout 120 --timeout-method thread" \
 "gpu_tests:600:python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread" \
 "bench_c1:200:python bench.py --config 1 --no-cpu-baseline" \
 "bench_c1_p1:200:OLPE_UNITS=1 python bench.py --config 1 --no-cpu-baseline --no-alt" \
 "bench:200:python bench.py --no-cpu-baseline" \
 "bench_c4:200:python bench.py --config 4 --no-cpu-baseline" \
 "bench_c4_p1:200:OLPE_UNITS=1 python bench.py --config 4 --no-cpu-baseline --no-alt"

export TMPDIR=/tmp
tools/gpu_steps.sh \
  "ring_test:240:python -u -m pytest tests/test_gpu_parity.py -x -v -k 'ring_sampler or bench_3source_128 or 128-2-fast' --timeout 60 --timeout-method thread" \
  "gpu_tests:400:python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread" \
  "ab_c4:300:AB_ARGS='--config 4' tools/ab_env.sh OLPE_RING=0"

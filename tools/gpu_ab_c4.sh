export TMPDIR=/tmp
tools/gpu_steps.sh \
  "gpu_tests:400:python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread" \
  "ab_c4:300:AB_ARGS='--config 4' tools/ab_libs.sh prev" \
  "ab_c2:300:tools/ab_libs.sh prev" \
  "post_c4:300:python tests/posterior_parity.py --config 4 --walkers 48 --iters 5000 --burn 1000"

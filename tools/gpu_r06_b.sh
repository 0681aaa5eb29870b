#!/bin/bash
# Round 6, second session: the communicator without the helper-thread join (direct,
# non-blocking RCCL set-up), then the whole GPU suite and smoke.
mkdir -p gpurun_out/r06b
tools/gpu_steps.sh \
  "r06b/comm:400:python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k 'rccl or comm_calls' tests/test_bench_gpu.py" \
  "r06b/gpu_tests:900:python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread" \
  "r06b/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'"

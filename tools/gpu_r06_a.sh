#!/bin/bash
# Round 6, first session: the new collective protocol (non-blocking RCCL communicator,
# poisoned check words, both moments rounds always entered, bounded waits), the 3-source
# exchange, the hand-off hold hook -- then the whole GPU suite and smoke.
mkdir -p gpurun_out/r06a
tools/gpu_steps.sh \
  "r06a/comm:300:python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k 'rccl' tests/test_bench_gpu.py" \
  "r06a/handoff:400:python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_gpu_long_reference.py -k handoffs" \
  "r06a/gpu_tests:900:python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread" \
  "r06a/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'"

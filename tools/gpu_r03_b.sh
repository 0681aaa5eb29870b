#!/bin/bash
# Round 3 session b: GPU tests (non-finite pixels, device moments, CLI posterior summary,
# bench exchange with one rank), the step-3 loader timing at 4,096 x 2,000 rows, and the
# roofline profiling session (tools/roofline_session.sh), then the default bench.
export TMPDIR=/tmp
df -h /tmp | tail -1
tools/gpu_steps.sh \
  "gpu_tests:600:python -u -m pytest tests -x -q -m gpu -rf --timeout 240 --timeout-method thread" \
  "smoke:120:python __graft_entry__.py smoke" \
  "loader_timing:400:python tools/loader_timing.py" && \
tools/roofline_session.sh r03 && \
tools/gpu_steps.sh "bench:300:python bench.py"

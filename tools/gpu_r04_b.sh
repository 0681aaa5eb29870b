#!/bin/bash
# Round 4, second GPU session: the whole GPU suite, then the round-4 roofline session
# (tools/roofline_session.sh r04: every bench shape at its SURVEY 8(d) default, incl.
# configs[1] at 1,000-iteration launches with the chain recorded every iteration).
mkdir -p gpurun_out/r04b
tools/gpu_steps.sh \
  "r04b/gpu_tests:500:python -u -m pytest tests -m gpu -x -q -rA --timeout 200 --timeout-method thread -p no:cacheprovider" \
  || exit $?
tools/roofline_session.sh r04 fast c1_fast c4_fast exact

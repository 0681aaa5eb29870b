#!/bin/bash
# (ran on commit 9dd5aa9, whose library had the 16-wave ring; it was removed after this
# measurement -- DESIGN.md §9 item 2 -- so OLPE_RING=16 is refused by later trees)
# Round 5: the 16-wave ring sampler (OLPE_RING=16) -- its tests, then a same-box A/B of
# configs[4] against the 12-wave ring (alternating, twice each).
mkdir -p gpurun_out/r05r16
B="python bench.py --config 4 --no-cpu-baseline --no-alt --no-csv"
tools/gpu_steps.sh \
  "r05r16/tests:600:python -u -m pytest tests -x -v -m gpu -k 'ring or long or c128' --timeout 300 --timeout-method thread" \
  "r05r16/ab_12a:200:OLPE_RING=12 $B" \
  "r05r16/ab_16a:200:OLPE_RING=16 $B" \
  "r05r16/ab_12b:200:OLPE_RING=12 $B" \
  "r05r16/ab_16b:200:OLPE_RING=16 $B"

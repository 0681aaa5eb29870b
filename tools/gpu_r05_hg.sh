#!/bin/bash
# Round 5: the one-slot (16-wave) sampler's shape-table rows through the scalar cache.
# diag/hgonly: -DOLPE_EXP_HG_ONLY (every row by scalar load, versions sized generously,
# no LDS fallback).  Its bit-equality tests against the 12-wave sampler, then a same-box
# A/B of configs[2] and configs[1] against the committed product (diag/base, built by
# tools/build_rev.sh HEAD base: rows from LDS) and the library with versions + LDS
# fallback (the working tree's product), alternating, twice.
mkdir -p gpurun_out/r05hg
B="python bench.py --no-cpu-baseline --no-alt --no-csv"
L="OLPE_LIB=diag/hgonly/libolpe.so"
K="OLPE_LIB=diag/base/libolpe.so"
tools/gpu_steps.sh \
  "r05hg/tests_hgonly:600:$L python -u -m pytest tests -x -v -m gpu -k 'sixteen_wave or bench_size or whole_ensemble or long_chains_match' --timeout 300 --timeout-method thread" \
  "r05hg/base_1:200:$K $B" \
  "r05hg/hgonly_1:200:$L $B" \
  "r05hg/prod_1:200:$B" \
  "r05hg/base_2:200:$K $B" \
  "r05hg/hgonly_2:200:$L $B" \
  "r05hg/prod_2:200:$B" \
  "r05hg/c1_base:200:$K $B --config 1" \
  "r05hg/c1_hgonly:200:$L $B --config 1"

#!/bin/bash
# Round 5: bound for shape-table rows read through the scalar cache (OLPE_DIAG_HSMEM:
# rows from constant global memory by s_load, results meaningless) against the product
# and against no per-row reads at all (OLPE_DIAG_HCONST).  Same box, alternating, twice.
B="python bench.py --no-cpu-baseline --no-alt --no-csv --steps 20 --warmup 5"
mkdir -p gpurun_out/r05hs
steps=()
for rep in 1 2; do
  steps+=("r05hs/base_$rep:200:$B")
  for v in hsmem hconst; do steps+=("r05hs/${v}_$rep:200:OLPE_LIB=diag/$v/libolpe.so $B"); done
done
tools/gpu_steps.sh "${steps[@]}"

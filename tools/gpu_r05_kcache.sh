#!/bin/bash
# Round 5: what bounds scalar-loaded shape-table rows -- the scalar cache's capacity or
# its cold misses.  Diagnostic builds (results meaningless, the same FP64 instructions):
# hsmem = one table shared by every wave (the +9.6 % bound), pw = a 1 KiB table per wave
# slot, pwhalf = 512 B per wave slot (the size of a mirrored half table, rows k and
# 2 kc + 1 - k share their values), pwrot / pwhalfrot = a fresh version every sweep.
# Same box, alternating, twice, against the product.
B="python bench.py --no-cpu-baseline --no-alt --no-csv --steps 20 --warmup 5"
mkdir -p gpurun_out/r05k
steps=()
for rep in 1 2; do
  steps+=("r05k/base_$rep:200:$B")
  for v in hsmem pw pwhalf pwrot pwhalfrot; do
    steps+=("r05k/${v}_$rep:200:OLPE_LIB=diag/$v/libolpe.so $B")
  done
done
tools/gpu_steps.sh "${steps[@]}"

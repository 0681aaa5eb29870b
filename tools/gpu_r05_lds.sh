#!/bin/bash
# Round 5: how much of configs[2]'s step the LDS reads of its sweep cost.  Diagnostic
# builds (results meaningless) with the same FP64 instructions: OLPE_DIAG_HCONST reads
# the shape-table rows once instead of per row (64 -> 4 LDS reads per sweep),
# OLPE_DIAG_DWCONST the cutout rows likewise.  Same box, alternating, twice; the clock by
# GRBM_GUI_ACTIVE for each.
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-alt --no-csv --steps 20 --warmup 5"
mkdir -p gpurun_out/r05lds
steps=()
for rep in 1 2; do
  steps+=("r05lds/base_$rep:200:$B")
  for v in hconst dwconst; do steps+=("r05lds/${v}_$rep:200:OLPE_LIB=diag/$v/libolpe.so $B"); done
done
for v in base hconst dwconst; do
  L=""; [ "$v" != base ] && L="OLPE_LIB=diag/$v/libolpe.so"
  steps+=("r05lds/clk_$v:200:$L timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/r05lds/clk_$v -o run --output-format csv -- $B")
done
tools/gpu_steps.sh "${steps[@]}"

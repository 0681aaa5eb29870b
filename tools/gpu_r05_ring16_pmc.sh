#!/bin/bash
# (ran on commit 9dd5aa9, whose library had the 16-wave ring; it was removed after this
# measurement -- DESIGN.md §9 item 2 -- so OLPE_RING=16 is refused by later trees)
# Round 5: VALU / FP64 counts and the held clock of the 12- and 16-wave rings (configs[4]),
# one box, the library with both (the 16-wave ring was measured, then removed).
export TMPDIR=/tmp
V="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"
B="python bench.py --config 4 --no-cpu-baseline --no-alt --no-csv"
mkdir -p gpurun_out/r05_ring16
for rg in 12 16; do
  d=gpurun_out/r05_ring16/w${rg}_1
  tools/gpu_steps.sh \
    "r05_ring16/bench_w${rg}_1:200:OLPE_RING=$rg $B --steps 5 --warmup 2" \
    "r05_ring16/prof_w${rg}_1:200:OLPE_RING=$rg rocprofv3 --kernel-trace --stats -d $d/prof -o run --output-format csv -- $B --steps 5 --warmup 2" \
    "r05_ring16/valu_w${rg}_1:200:OLPE_RING=$rg timeout -s KILL 180 rocprofv3 --pmc $V -d $d/valu -o run --output-format csv -- $B --steps 3 --warmup 1" \
    || exit $?
done

#!/bin/bash
# Verdict r04 item 4: bound the configs[4] ring sampler's 4-waves-per-SIMD lever before
# building it.  One session, one box, one library (diag/ring8: tools/diag_build.sh ring8
# -DOLPE_DIAG_RING8, the 12-wave kernel as in the product plus the same sweep at 8 waves
# per workgroup, 2 per SIMD, with the 12-wave register budget): per wave count, the bench
# line (HIP-event kernel ms), rocprofv3 kernel stats and the SQ VALU / clock counters.
# Summarised here by tools/ring8_summary.py into profiles/r05/ring8/.
export TMPDIR=/tmp
L=diag/ring8/libolpe.so
V="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"
B="python bench.py --config 4 --no-cpu-baseline --no-alt --no-csv"
mkdir -p gpurun_out/r05_ring8
for rep in 1 2; do
for rg in 12 8; do
  d=gpurun_out/r05_ring8/w${rg}_$rep
  tools/gpu_steps.sh \
    "r05_ring8/bench_w${rg}_$rep:200:OLPE_LIB=$L OLPE_RING=$rg $B --steps 5 --warmup 2" \
    "r05_ring8/prof_w${rg}_$rep:200:OLPE_LIB=$L OLPE_RING=$rg rocprofv3 --kernel-trace --stats -d $d/prof -o run --output-format csv -- $B --steps 5 --warmup 2" \
    "r05_ring8/valu_w${rg}_$rep:200:OLPE_LIB=$L OLPE_RING=$rg timeout -s KILL 180 rocprofv3 --pmc $V -d $d/valu -o run --output-format csv -- $B --steps 3 --warmup 1" \
    || exit $?
done
done

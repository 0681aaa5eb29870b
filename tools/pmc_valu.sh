#!/bin/bash
# SQ VALU instruction mix of the sampler kernel for one bench config/mode (one
# rocprofv3 pass, 5 SQ counters), summarised into profiles/valu_counts.json:
#   tools/pmc_valu.sh <config> <mode> <tag>
export TMPDIR=/tmp
cfg=${1:-2}; mode=${2:-fast}; tag=${3:-r02}
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt --mode $mode --config $cfg"
key=$mode; [ "$cfg" != "2" ] && key="c${cfg}_$mode"
case $cfg in 1) steps=409600;; 2) steps=6553600;; 4) steps=1638400;; esac
d=gpurun_out/pmc_${tag}_valu_$key
tools/gpu_steps.sh \
  "valu_$key:200:rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 -d $d -o run --output-format csv -- $B" \
  && python tools/pmc_valu.py "$key" "$d" "$steps"

#!/bin/bash
# SQ instruction / cycle counters of the sampler kernel, three separate rocprofv3 passes.
export TMPDIR=/tmp
mode=${1:-fast}
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt --mode $mode"
tools/gpu_steps.sh \
  "sqA_$mode:200:rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d gpurun_out/sqA_$mode -o run --output-format csv -- $B" \
  "sqB_$mode:200:rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_INT32 -d gpurun_out/sqB_$mode -o run --output-format csv -- $B" \
  "sqC_$mode:200:rocprofv3 --pmc SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FLOPS_FP64 GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM SQ_INSTS_BRANCH -d gpurun_out/sqC_$mode -o run --output-format csv -- $B"

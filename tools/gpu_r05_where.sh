#!/bin/bash
# Round 5: where a 16-wave configs[2] step goes on the final tree -- SQ wave-state and
# instruction counters of the product (two rocprofv3 passes, tools/pmc_sq_cfg.sh) and the
# per-section cycle split of the diagnostic OLPE_DIAG_TIMING build (tools/diag_timing.py;
# built by tools/diag_build.sh timing -DOLPE_DIAG_TIMING); the same for configs[4]'s ring.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05w
timeout -k 10 500 tools/pmc_sq_cfg.sh 2 > gpurun_out/r05w/sq_c2.log 2>&1 && \
  mv gpurun_out/sqB_c2 gpurun_out/sqD_c2 gpurun_out/r05w/ && \
timeout -k 10 500 tools/pmc_sq_cfg.sh 4 > gpurun_out/r05w/sq_c4.log 2>&1 && \
  mv gpurun_out/sqB_c4 gpurun_out/sqD_c4 gpurun_out/r05w/ && \
tools/gpu_steps.sh \
  "r05w/timing_c2:200:OLPE_LIB=diag/timing/libolpe.so python tools/diag_timing.py 65536 100 64 2" \
  "r05w/timing_c4:200:OLPE_LIB=diag/timing/libolpe.so OLPE_UNITS=1 python tools/diag_timing.py 3072 100 128 3"

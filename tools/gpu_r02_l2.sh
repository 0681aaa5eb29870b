#!/bin/bash
# L1 -> L2 read requests and L2 hits/misses per walker-step (configs[4] vs configs[2])
export TMPDIR=/tmp
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt"
tools/gpu_steps.sh \
  "l2_c4:120:rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/pmc_r02_l2_c4 -o run --output-format csv -- $B --config 4" \
  "l2_c2:120:rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/pmc_r02_l2_c2 -o run --output-format csv -- $B --config 2"

#!/bin/bash
# PMC traffic passes for configs[4] exact and configs[1] (fast, exact); kernel stats for configs[1].
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-alt"
tools/gpu_steps.sh \
 "pmc_fetch_c4x:120:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_r01_fetch_c4_exact -o run --output-format csv -- $B --config 4 --mode exact" \
 "pmc_write_c4x:120:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_r01_write_c4_exact -o run --output-format csv -- $B --config 4 --mode exact" \
 "prof_c1:120:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01_c1_fast -o run --output-format csv -- $B --config 1" \
 "pmc_fetch_c1:120:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_r01_fetch_c1_fast -o run --output-format csv -- $B --config 1" \
 "pmc_write_c1:120:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_r01_write_c1_fast -o run --output-format csv -- $B --config 1" \
 "pmc_fetch_c1x:120:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_r01_fetch_c1_exact -o run --output-format csv -- $B --config 1 --mode exact" \
 "pmc_write_c1x:120:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_r01_write_c1_exact -o run --output-format csv -- $B --config 1 --mode exact"

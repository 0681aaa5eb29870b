#!/bin/bash
# Round-2 profile refresh on the current kernels: kernel stats (c2 fast/exact, c1, c4),
# PMC FETCH/WRITE traffic per config, full bench lines.
export TMPDIR=/tmp
tag=r02
B="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-alt"
tools/gpu_steps.sh \
  "bench:300:python bench.py" \
  "prof_fast:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_fast -o run --output-format csv -- $B --mode fast" \
  "prof_exact:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_exact -o run --output-format csv -- $B --mode exact" \
  "prof_c1:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_c1_fast -o run --output-format csv -- python bench.py --config 1 --no-cpu-baseline --no-alt" \
  "prof_c4:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_c4_fast -o run --output-format csv -- $B --config 4" \
  "pmc_fetch_fast:120:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${tag}_fetch_fast -o run --output-format csv -- $B --mode fast" \
  "pmc_write_fast:120:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${tag}_write_fast -o run --output-format csv -- $B --mode fast" \
  "pmc_fetch_exact:120:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${tag}_fetch_exact -o run --output-format csv -- $B --mode exact" \
  "pmc_write_exact:120:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${tag}_write_exact -o run --output-format csv -- $B --mode exact" \
  "pmc_fetch_c1:120:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${tag}_fetch_c1_fast -o run --output-format csv -- $B --config 1" \
  "pmc_write_c1:120:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${tag}_write_c1_fast -o run --output-format csv -- $B --config 1" \
  "pmc_fetch_c4:120:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${tag}_fetch_c4_fast -o run --output-format csv -- $B --config 4" \
  "pmc_write_c4:120:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${tag}_write_c4_fast -o run --output-format csv -- $B --config 4" \
  "bench_c1:300:python bench.py --config 1" \
  "bench_c4:300:python bench.py --config 4"

#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel stats, PMC traffic passes.
# usage: tools/gpu_session.sh <round-tag> [skip-tests]
tag=${1:-r01}
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-alt"
T="gpu_tests:900:python -u -m pytest tests -q -m gpu -rf --timeout 300 --timeout-method thread"
[ "$2" = "skip-tests" ] && T="noop:10:true"
tools/gpu_steps.sh \
  "$T" \
  "bench:400:python bench.py" \
  "prof_fast:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_fast -o run --output-format csv -- $B --mode fast" \
  "prof_exact:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_exact -o run --output-format csv -- $B --mode exact" \
  "pmc_fetch_fast:300:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${tag}_fetch_fast -o run --output-format csv -- $B --mode fast" \
  "pmc_write_fast:300:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${tag}_write_fast -o run --output-format csv -- $B --mode fast" \
  "pmc_fetch_exact:300:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${tag}_fetch_exact -o run --output-format csv -- $B --mode exact" \
  "pmc_write_exact:300:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${tag}_write_exact -o run --output-format csv -- $B --mode exact" \
  "prof_c4:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_c4_fast -o run --output-format csv -- $B --config 4" \
  "pmc_fetch_c4:300:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${tag}_fetch_c4_fast -o run --output-format csv -- $B --config 4" \
  "pmc_write_c4:300:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${tag}_write_c4_fast -o run --output-format csv -- $B --config 4" \
  "bench_c4:300:python bench.py --config 4" \
  "prof_c1:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_c1_fast -o run --output-format csv -- $B --config 1" \
  "bench_c1:300:python bench.py --config 1"

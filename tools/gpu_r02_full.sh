#!/bin/bash
# Round-2 full refresh on HEAD: GPU tests + smoke, SQ VALU counts (fast, exact, c1, c4),
# PMC FETCH/WRITE traffic (c2 fast/exact, c1, c4), L2 counters (c4), rocprofv3 kernel
# stats (c2 fast/exact, c1, c4) and the bench lines (default, --config 1, --config 4).
# Summaries are made locally from gpurun_out/ (tools/pmc_valu.py, tools/pmc_summary.py).
export TMPDIR=/tmp
tag=${1:-r02f}
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt"
S="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-alt"
V="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"
tools/gpu_steps.sh \
  "gpu_tests:400:python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread" \
  "smoke:120:python __graft_entry__.py smoke" \
  "valu_fast:150:rocprofv3 --pmc $V -d gpurun_out/pmc_${tag}_valu_fast -o run --output-format csv -- $B --mode fast" \
  "valu_exact:200:rocprofv3 --pmc $V -d gpurun_out/pmc_${tag}_valu_exact -o run --output-format csv -- $B --mode exact" \
  "valu_c1:150:rocprofv3 --pmc $V -d gpurun_out/pmc_${tag}_valu_c1_fast -o run --output-format csv -- $B --config 1" \
  "valu_c4:150:rocprofv3 --pmc $V -d gpurun_out/pmc_${tag}_valu_c4_fast -o run --output-format csv -- $B --config 4" \
  "fetch_fast:120:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${tag}_fetch_fast -o run --output-format csv -- $B --mode fast" \
  "write_fast:120:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${tag}_write_fast -o run --output-format csv -- $B --mode fast" \
  "fetch_exact:200:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${tag}_fetch_exact -o run --output-format csv -- $B --mode exact" \
  "write_exact:200:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${tag}_write_exact -o run --output-format csv -- $B --mode exact" \
  "fetch_c1:120:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${tag}_fetch_c1_fast -o run --output-format csv -- $B --config 1" \
  "write_c1:120:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${tag}_write_c1_fast -o run --output-format csv -- $B --config 1" \
  "fetch_c4:120:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${tag}_fetch_c4_fast -o run --output-format csv -- $B --config 4" \
  "write_c4:120:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${tag}_write_c4_fast -o run --output-format csv -- $B --config 4" \
  "l2_c4:120:rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/pmc_${tag}_l2_c4 -o run --output-format csv -- $B --config 4" \
  "prof_fast:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_fast -o run --output-format csv -- $S --mode fast" \
  "prof_exact:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_exact -o run --output-format csv -- $S --mode exact" \
  "prof_c1:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_c1_fast -o run --output-format csv -- python bench.py --config 1 --no-cpu-baseline --no-alt" \
  "prof_c4:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_c4_fast -o run --output-format csv -- $S --config 4" \
  "bench:300:python bench.py" \
  "bench_c1:300:python bench.py --config 1" \
  "bench_c4:300:python bench.py --config 4"

#!/bin/bash
# Round 3 final session on one box: GPU tests + smoke, the roofline profiling session
# (tools/roofline_session.sh: rocprofv3 kernel trace + stats, SQ VALU + clock, HBM
# FETCH/WRITE for every bench shape, summarised on the box into profiles/ so that the
# bench lines after it read this session's counts; rerun the summary here after the
# merge to commit the same files), the bench lines (configs[2] default, [1], [4]) and
# a 2-rank launcher rehearsal sharing the one GPU.
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "gpu_tests:700:python -u -m pytest tests -q -m gpu -rf --timeout 240 --timeout-method thread" \
  "smoke:120:python __graft_entry__.py smoke" && \
tools/roofline_session.sh r03 && \
for k in fast exact c1_fast c4_fast; do python tools/roofline_summary.py r03 $k gpurun_out/r03_$k || exit 1; done && \
tools/gpu_steps.sh \
  "bench:300:python bench.py" \
  "bench_c1:300:python bench.py --config 1" \
  "bench_c4:300:python bench.py --config 4" \
  "bench_exchange:300:python bench.py --exchange --verify-exchange --no-cpu-baseline --no-alt" \
  "dist2_share:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --share-gpu --steps 5 --warmup 1"

#!/bin/bash
# Round 5, the roofline session on the final tree (verdict r04 item 6:
# tools/roofline_session.sh r05, every bench shape at its SURVEY 8(d) default, the
# kernel stats now listing fold_rows_kernel / fold_cols_kernel), then each config's bench
# line with the CPU baselines and the 2-rank rehearsal, on the same box.
mkdir -p gpurun_out/r05f
tools/roofline_session.sh r05 fast c1_fast c4_fast exact || exit $?
tools/gpu_steps.sh \
  "r05f/bench:300:python bench.py" \
  "r05f/bench_c1:300:python bench.py --config 1" \
  "r05f/bench_c4:300:python bench.py --config 4" \
  "r05f/bench_c0:300:python bench.py --config 0" \
  "r05f/bench_exchange:300:python bench.py --exchange --verify-exchange --no-cpu-baseline --no-alt" \
  "r05f/bench_gpus2_share:300:python bench.py --gpus 2 --share-gpu --no-cpu-baseline --no-alt"

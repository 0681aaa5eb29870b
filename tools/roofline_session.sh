#!/bin/bash
# One profiling session for bench.py's roofline (round 3): for every bench shape, in
# the same session on the same box,
#   prof_<key>  rocprofv3 --kernel-trace --stats of a bench run (its JSON line carries
#               the HIP-event kernel_ms of the same dispatches)
#   valu_<key>  rocprofv3 --pmc: SQ VALU mix (FP64 lane-ops) + GRBM_GUI_ACTIVE (clock)
#   fetch/write rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, HBM bytes)
# then (here, after gpurun merged gpurun_out/) tools/roofline_summary.py copies the
# files into profiles/<tag>/, writes profiles/<tag>/roofline.json and refreshes
# profiles/valu_counts.json / pmc_traffic.json, so that the frac of the session is
# recomputable from the committed files.
#   tools/roofline_session.sh <tag> [keys...]    (keys: fast exact c1_fast c4_fast)
export TMPDIR=/tmp
tag=${1:-r04}; shift
keys=${*:-"fast exact c1_fast c4_fast"}
for key in $keys; do
  case $key in
    # (round 4: each config's bench defaults -- SURVEY 8(d)'s iterations and stride)
    fast) cfg=2; mode=fast; steps=20; warm=5;;
    exact) cfg=2; mode=exact; steps=4; warm=1;;
    c1_fast) cfg=1; mode=fast; steps=10; warm=2;;
    c4_fast) cfg=4; mode=fast; steps=5; warm=2;;
    *) echo "unknown key $key"; exit 2;;
  esac
  B="python bench.py --config $cfg --mode $mode --no-cpu-baseline --no-alt"
  V="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"
  d=gpurun_out/${tag}_$key
  tools/gpu_steps.sh \
    "prof_${tag}_$key:300:rocprofv3 --kernel-trace --stats -d $d/prof -o run --output-format csv -- $B --steps $steps --warmup $warm" \
    "valu_${tag}_$key:200:timeout -s KILL 180 rocprofv3 --pmc $V -d $d/valu -o run --output-format csv -- $B --steps 3 --warmup 1" \
    "fetch_${tag}_$key:200:timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $d/fetch -o run --output-format csv -- $B --steps 3 --warmup 1" \
    "write_${tag}_$key:200:timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $d/write -o run --output-format csv -- $B --steps 3 --warmup 1" \
    || exit $?
  cp gpurun_out/prof_${tag}_$key.log $d/bench_line.log
done

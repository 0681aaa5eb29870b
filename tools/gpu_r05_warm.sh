#!/bin/bash
# Round 5: the DVFS ramp and the bench's warm-up -- each config's default line (§8(d)'s
# timed launches after its short default warm-up) against the same timed launches after
# ~0.5 s of warm-up launches, same box, alternating, twice; the SMU clock in each line.
B="python bench.py --no-cpu-baseline --no-alt --no-csv"
mkdir -p gpurun_out/r05w2
steps=()
for rep in 1 2; do
  steps+=("r05w2/c2_def_$rep:200:$B" "r05w2/c2_w40_$rep:200:$B --warmup 40")
  steps+=("r05w2/c1_def_$rep:200:$B --config 1" "r05w2/c1_w60_$rep:200:$B --config 1 --warmup 60")
  steps+=("r05w2/c4_def_$rep:200:$B --config 4" "r05w2/c4_w35_$rep:200:$B --config 4 --warmup 35")
done
tools/gpu_steps.sh "${steps[@]}"

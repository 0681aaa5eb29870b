#!/bin/bash
# Round 5: the shape-table rows two blocks ahead in the 12-wave 64x64 sampler, where 21
# VGPRs are free (diag/h2, -DOLPE_EXP_H2), against the product's 12-wave sampler
# (OLPE_WPB=12) and its 16-wave default, configs[2], same box, alternating, twice; then
# the 12-wave bit-equality tests with the experiment.
B="python bench.py --no-cpu-baseline --no-alt --no-csv"
L="OLPE_LIB=diag/h2/libolpe.so"
mkdir -p gpurun_out/r05h2
steps=()
for rep in 1 2; do
  steps+=("r05h2/p16_$rep:200:$B" "r05h2/p12_$rep:200:OLPE_WPB=12 $B" "r05h2/h2_12_$rep:200:$L OLPE_WPB=12 $B")
done
steps+=("r05h2/tests:400:$L python -u -m pytest tests -v -m gpu -k 'sixteen_wave or bench_size' --timeout 300 --timeout-method thread")
tools/gpu_steps.sh "${steps[@]}"

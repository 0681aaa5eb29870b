#!/bin/bash
# Round 4: the one-wave-per-walker moment fold -- the tests that check moments, then the
# fold's time in a kernel trace of configs[1] (557 MB of stride-1 rows per launch) and
# configs[2] (89 MB), and the bench lines.
export TMPDIR=/tmp
mkdir -p gpurun_out/r04fold
tools/gpu_steps.sh \
  "r04fold/tests:400:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_whole_ensembles.py tests/test_cli_gpu.py -x -q -k 'moments or configs1 or rccl or shards or posterior or summary' --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "r04fold/prof_c1:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04fold/prof_c1 -o run --output-format csv -- python bench.py --config 1 --no-cpu-baseline --no-alt" \
  "r04fold/prof_c2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04fold/prof_c2 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-alt"

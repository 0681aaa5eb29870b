#!/bin/bash
# configs[1] with CLI-shaped launches: apf_step2 at 4,096 walkers and the default 1 GiB
# --mem-budget launches ~1,920 iterations at stride 1 (step2.chunk_size); the bench's
# default configs[1] step is 100 iterations.  Same box, one after the other.
B="python bench.py --config 1 --no-cpu-baseline --no-alt"
tools/gpu_steps.sh \
  "c1_100:200:$B" \
  "c1_1920_s1:200:$B --iters 1920 --stride 1 --steps 20 --warmup 3" \
  "c1_1920_s10:200:$B --iters 1920 --stride 10 --steps 20 --warmup 3" \
  "c2_100:200:python bench.py --no-cpu-baseline --no-alt"

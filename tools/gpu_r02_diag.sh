#!/bin/bash
P='import json,sys; d=json.loads(sys.stdin.readline()); print(round(d["value"]/1e6,1), "M  kernel_ms", round(d["roofline"]["kernel_ms"],3), "ms_per_step", round(d["ms_per_step"],3))'
for wu in 2 20 100 400; do
  echo "c1 warmup $wu steps 100: $(timeout -k 10 120 python bench.py --config 1 --no-cpu-baseline --no-alt --warmup $wu --steps 100 | python -c "$P")" >> gpurun_out/warmup_c1.log || exit 1
done
for wu in 2 20; do
  echo "c2 warmup $wu steps 20: $(timeout -k 10 120 python bench.py --no-cpu-baseline --no-alt --warmup $wu --steps 20 | python -c "$P")" >> gpurun_out/warmup_c1.log || exit 1
done

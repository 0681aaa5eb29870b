#!/bin/bash
P='import json,sys; d=json.loads(sys.stdin.readline()); print(round(d["value"]/1e6,1), "M  kernel_ms", round(d["roofline"]["kernel_ms"],2))'
for rep in 1 2; do
for it in 100 300 1000 3000; do
  st=$((1000 / it)); [ $st -lt 3 ] && st=3
  echo "iters $it steps $st: $(timeout -k 10 200 python bench.py --no-cpu-baseline --no-alt --iters $it --steps $st --warmup 1 | python -c "$P")" >> gpurun_out/iters_ab.log || exit 1
done
done

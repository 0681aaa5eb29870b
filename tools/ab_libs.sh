#!/bin/bash
# A/B the product library against diagnostic variants on one box:
#   [AB_ARGS="--mode exact"] tools/ab_libs.sh name1 name2 ...
B="python bench.py --no-cpu-baseline --no-alt --steps 8 $AB_ARGS"
P='import json,sys; d=json.loads(sys.stdin.readline()); print(round(d["value"]/1e6,1), "M  kernel_ms", round(d["roofline"]["kernel_ms"],2))'
for rep in 1 2; do
  echo "base $($B | python -c "$P")"
  for v in "$@"; do
    echo "$v $(OLPE_LIB=diag/$v/libolpe.so $B | python -c "$P")"
  done
done

#!/bin/bash
# A/B the product library under environment variants and diagnostic libraries:
#   [AB_ARGS="--config 4"] tools/ab_env.sh "NAME=VAL ..." diag:<name> ...
B="python bench.py --no-cpu-baseline --no-alt --steps 8 $AB_ARGS"
P='import json,sys; d=json.loads(sys.stdin.readline()); print(round(d["value"]/1e6,1), "M  kernel_ms", round(d["roofline"]["kernel_ms"],2))'
for rep in 1 2; do
  echo "base $($B | python -c "$P")"
  for v in "$@"; do
    if [[ $v == diag:* ]]; then
      echo "$v $(OLPE_LIB=diag/${v#diag:}/libolpe.so $B | python -c "$P")"
    else
      echo "$v $(env $v $B | python -c "$P")"
    fi
  done
done

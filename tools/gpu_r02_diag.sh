#!/bin/bash
for cfg in "3072 100 1" "4096 100 3" "65536 100 1"; do
  for env in "OLPE_BALANCE=0 OLPE_STAGGER=0" "OLPE_BALANCE=0 OLPE_STAGGER=4" "OLPE_BALANCE=0 OLPE_STAGGER=8" "OLPE_BALANCE=0 OLPE_STAGGER=16" "OLPE_BALANCE=1 OLPE_STAGGER=0" "OLPE_BALANCE=1 OLPE_STAGGER=8"; do
    echo "== $env" >> gpurun_out/span_diag2.log
    env $env OLPE_LIB=diag/span/libolpe.so timeout -k 10 120 python tools/span_diag.py $cfg >> gpurun_out/span_diag2.log 2>&1 || exit 1
  done
done

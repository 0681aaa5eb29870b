#!/bin/bash
# long-run posterior parity through the chunked (work-unit) path
OLPE_UNITS=4 timeout -k 10 600 python tests/posterior_parity.py --walkers 16 --iters 20000 --burn 2000 > gpurun_out/posterior_parity_units.log 2>&1

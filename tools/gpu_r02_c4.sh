#!/bin/bash
AB_ARGS="--config 4" timeout -k 10 400 tools/ab_libs.sh gw4 > gpurun_out/ab_c4_gw4.log 2>&1

#!/bin/bash
# Round 5: tools/gpu_r05_a.sh (suite, default bench line, 2-rank rehearsal), then the
# configs[4] 8- vs 12-wave ring session (tools/gpu_r05_ring8.sh), in one box call.
tools/gpu_r05_a.sh && tools/gpu_r05_ring8.sh

#!/bin/bash
# SQ cycle counters of the sampler kernel for one bench config (one rocprofv3 pass):
#   tools/pmc_sq_cfg.sh <config> [mode]
export TMPDIR=/tmp
cfg=${1:-2}; mode=${2:-fast}
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt --mode $mode --config $cfg"
tools/gpu_steps.sh \
  "sqB_c$cfg:200:rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d gpurun_out/sqB_c$cfg -o run --output-format csv -- $B" \
  "sqD_c$cfg:200:rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/sqD_c$cfg -o run --output-format csv -- $B"
python - "$cfg" <<'PY'
import csv, collections, sys
cfg = sys.argv[1]
for p in ("sqB", "sqD"):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/{p}_c{cfg}/run_counter_collection.csv")):
        if "gibbs" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(p, {k: f"{sum(v)/len(v):.4g}" for k, v in acc.items()})
PY

#!/bin/bash
# Summarise a tools/gpu_r02_full.sh run (gpurun_out/) into profiles/: VALU counts
# (profiles/valu_counts.json), PMC traffic (profiles/pmc_traffic.json), kernel stats,
# counter CSVs, bench lines, GPU test and smoke logs.  usage: tools/refresh_local.sh <tag> [dir]
T=${1:-r02g}; P=${2:-profiles/r02}
for k in "fast 6553600" "exact 6553600" "c1_fast 409600" "c4_fast 1638400"; do
  set -- $k
  python tools/pmc_valu.py $1 gpurun_out/pmc_${T}_valu_$1 $2 > /dev/null || exit 1
done
for m in fast exact c1_fast c4_fast; do
  python tools/pmc_summary.py $m gpurun_out/pmc_${T}_fetch_$m gpurun_out/pmc_${T}_write_$m > /dev/null || exit 1
  cp gpurun_out/prof_${T}_$m/run_kernel_stats.csv $P/kernel_stats_$m.csv
  cp gpurun_out/pmc_${T}_valu_$m/run_counter_collection.csv $P/pmc_valu_$m.csv
  cp gpurun_out/pmc_${T}_fetch_$m/run_counter_collection.csv $P/pmc_fetch_$m.csv
  cp gpurun_out/pmc_${T}_write_$m/run_counter_collection.csv $P/pmc_write_$m.csv
done
cp gpurun_out/pmc_${T}_l2_c4/run_counter_collection.csv $P/pmc_l2_c4_fast.csv
for f in bench bench_c1 bench_c4 gpu_tests smoke; do cp gpurun_out/$f.log $P/$f.log; done
tail -n 1 $P/gpu_tests.log; tail -n 1 $P/smoke.log
python - <<'PY'
import json
v = json.load(open("profiles/valu_counts.json"))
print({k: round(x["valu_per_step"], 1) for k, x in v.items()})
for f in ("bench", "bench_c1", "bench_c4"):
    d = json.loads(open(f"profiles/r02/{f}.log").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, round(d["value"] / 1e6, 1), "M", round(r["kernel_ms"], 3), "ms frac", round(r["frac"], 3),
          "issue", round(r["valu_issue_frac"], 3), "stale", r.get("counts_stale"),
          "cpu", round(d.get("cpu_baseline", {}).get("value", 0)))
PY

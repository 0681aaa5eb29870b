#!/bin/bash
# Per-variant walker-steps/s and SQ_INSTS_VALU per walker-step (one rocprofv3 pass each)
#   tools/ab_valu.sh name1 name2 ...   (diag/<name>/libolpe.so; "base" = product library)
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-alt --steps 3 --warmup 1"
for v in base "$@"; do
  if [ "$v" = base ]; then unset OLPE_LIB; else export OLPE_LIB=diag/$v/libolpe.so; fi
  rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/valu_$v -o run --output-format csv -- $B > gpurun_out/valu_$v.log 2>&1 || exit 1
  python - "$v" <<'PY'
import csv, collections, sys, json
v = sys.argv[1]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f"gpurun_out/valu_{v}/run_counter_collection.csv")):
    if "gibbs" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
val = [json.loads(l) for l in open(f"gpurun_out/valu_{v}.log") if l.startswith("{")][0]["value"]
print(v, f"{val/1e6:.1f} M/s", {k: round(sum(x)/len(x)/6.5536e6, 1) for k, x in acc.items()})
PY
done

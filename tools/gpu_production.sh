#!/bin/bash
# The reference's production setting end to end on one GPU: accept_min = 100000 (about
# 1.6 M iterations per walker, apf_step2.py:300; 1.9 M for three sources), burn_in 6000
# (0 for three sources, 3body/apf_step2_3body.py:37-38), an N x N synthetic frame of
# NSRC sources, W walkers, a chain row every STRIDE iterations; then step 3 on the chain
# files and from step 2's device moments, and the two summaries compared.
#   tools/gpu_production.sh [walkers] [stride] [n] [nsrc]
set -e
W=${1:-4096}; ST=${2:-2000}; N=${3:-64}; NS=${4:-2}
if [ "$NS" = 3 ]; then S2=3body/apf_step2_3body.py; S3=3body/apf_step3_3body.py; else S2=apf_step2.py; S3=apf_step3.py; fi
D=$(mktemp -d)
trap 'rm -rf "$D"' EXIT
P=$(python -c "import sys; sys.path.insert(0, '.'); from olpefit_amd import synth; print(synth.write_case('$D', $N, $NS))")
OUT=$(dirname "$P")/$(basename "$P" | cut -d. -f3)_apf_results
t0=$(date +%s.%N)
python -u $S2 "$P" --walkers $W --record-stride $ST --seed 1 --timing | grep --line-buffered -v "^Initial guess"   # progress lines: a long run is not silent
t1=$(date +%s.%N)
python - "$OUT" "$W" "$t0" "$t1" "$N" "$NS" <<'PY'
import json, os, sys
out, W, t0, t1 = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), float(sys.argv[4])
n, nsrc = sys.argv[5], sys.argv[6]
s = json.load(open(os.path.join(out, "posterior_summary.json")))
names = [k for k in s if not k.startswith("_") and "tries" in s[k]]
steps = sum(s[k]["tries"] for k in names)          # every walker's tries = its iterations
files = [f for f in os.listdir(out) if f.endswith("_finalarray_mpi.csv")]
size = sum(os.path.getsize(os.path.join(out, f)) for f in files)
print(f"step 2: {W} walkers, {n}x{n}, {nsrc} sources, accept_min 100000, burn_in "
      f"{6000 if nsrc == '2' else 0}: wall {t1 - t0:.1f} s "
      f"(process start, launches, chain files, checkpoints, summary)")
print(f"  iterations per walker {steps / W:.0f}, walker-steps {steps:.4e}: "
      f"{steps / (t1 - t0):.3e} walker-steps/s end to end")
print(f"  {len(files)} chain files, {size / 1e9:.2f} GB, {s['_rows_per_walker']} rows each")
print("  posterior means:", {k: round(s[k]["mean"], 6) for k in names[:4]},
      "GR RC max:", round(max(s[k]["gr_rc"] for k in names), 6))
PY
t2=$(date +%s.%N)
python $S3 "$P" synthetic -s $W -q > /dev/null
cp "$OUT/step3_summary.json" "$D/from_files.json"
t3=$(date +%s.%N)
python $S3 "$P" synthetic -s $W --from-moments -q > /dev/null
t4=$(date +%s.%N)
echo "step 3 from the chain files: $(python -c "print(round($t3 - $t2, 2))") s; from the moments: $(python -c "print(round($t4 - $t3, 2))") s"
python - "$D/from_files.json" "$OUT/step3_summary.json" <<'PY'
import json, sys
a, b = (json.load(open(p))["parameters"] for p in sys.argv[1:3])
rel = max(abs(a[k][q] - b[k][q]) / max(abs(a[k][q]), 1e-300)
          for k in a for q in ("mean", "std", "gr_rc") if q in a[k] and q in b[k])
print(f"step 3 from the files vs from the device moments: max relative difference {rel:.2e} "
      f"(mean, std, GR RC of {len(a)} parameters)")
PY

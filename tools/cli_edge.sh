#!/bin/bash
# odd CLI combinations (small): each must exit 0 and leave consistent files
set -e
export TMPDIR=/tmp
D=$(mktemp -d)
P=$(python -c "import sys; sys.path.insert(0, '.'); from olpefit_amd import synth; print(synth.write_case('$D', 32, 2))")
run() { echo "--- $*"; python apf_step2.py "$P" "$@" -q && ls $(dirname $P)/00001_apf_results | wc -l; }
run --walkers 1 --iters 5 --seed 3
run --walkers 2 --iters 25 --burn-in 100 --seed 3
run --walkers 3 --iters 57 --record-stride 7 --seed 3
run --walkers 3 --iters 40 --npy --no-csv --seed 3
run --walkers 5 --accept-min 3 --burn-in 0 --seed 3
run --walkers 4 --iters 30 --exact --fixed-bkgd --seed 3
run --walkers 4 --iters 30 --chunk 7 --checkpoint-every 1 --seed 3
# the last run's default burn-in leaves only the seed row: step 3 must say so, not trace back
if python apf_step3.py "$P" sys -s 4 -q > $D/s3.log 2>&1; then echo "step3 should have failed"; exit 1; fi
grep -q "none left after additional_burnin" $D/s3.log && echo step3-short-run-error-ok
run --walkers 4 --iters 30 --burn-in 0 --seed 3
python apf_step3.py "$P" sys -s 4 -q > /dev/null && echo step3-ok
P3=$(python -c "import sys; sys.path.insert(0, '.'); from olpefit_amd import synth; print(synth.write_case('$D/t', 33, 3))")
echo "--- 3body 33x33"; python 3body/apf_step2_3body.py "$P3" --walkers 3 --iters 50 --seed 1 -q && python 3body/apf_step3_3body.py "$P3" sys -s 3 -q > /dev/null && echo step3-3body-ok
rm -rf $D
echo ALL-OK

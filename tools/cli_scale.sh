#!/bin/bash
# End-to-end step 2 CLI at scale on the GPU box: synthetic 64x64 frame, W walkers,
# fixed length, chain files written by the native writer; prints the wall times.
#   tools/cli_scale.sh [walkers] [iters] [stride]
W=${1:-4096}; IT=${2:-2000}; ST=${3:-10}
D=$(mktemp -d)
python -c "import sys; sys.path.insert(0, '.'); from olpefit_amd import synth; print(synth.write_case('$D', 64, 2))" > $D/path
P=$(cat $D/path)
t0=$(date +%s.%N)
python apf_step2.py "$P" --walkers $W --iters $IT --burn-in 0 --record-stride $ST --seed 1 -q
t1=$(date +%s.%N)
echo "step 2 CLI wall: $(python -c "print(round($t1 - $t0, 2))") s for $W walkers x $IT iterations (stride $ST)"
OUT=$(dirname "$P")/$(basename "$P" | cut -d. -f3)_apf_results
echo "files: $(ls $OUT | wc -l), bytes: $(du -sb $OUT | cut -f1)"
python -c "
import sys; sys.path.insert(0, '.')
from olpefit_amd import step3
c = step3.load_chains('$OUT', $W, additional_burnin=1)
print('step-3 read:', c.shape)
"
rm -rf $D

#!/bin/bash
# Same-box A/B of an older round's whole tree against HEAD on the FFT-mode headline (VERDICT r05
# #2: is k_col2's drift across driver boxes box or code?).  The old tree is extracted and built
# in this container (git archive <commit> bench.py binary-hologram-reinforcement-learning_amd
# include oracle | tar -x -C _ab/<tag>; make -C its csrc); each tree runs its OWN bench.py and
# library, alternated REPS times.  Run ON the GPU box from the repo root:
#   bash tools/ab_rounds.sh TAG _ab/r03l [REPS]
set -o pipefail
T=$1; OLD=$2; REPS=${3:-3}
mkdir -p gpurun_out/$T
NEW_Q="--steps 20 --warmup 3 --no-psf --no-ppo --no-probe --no-precision --no-obs --dbs-flips 0 --cpu-sample 0 --no-psnr-check --no-planes --no-crop --no-dropin --no-scipy"
OLD_Q="--steps 20 --warmup 3 --no-psf --no-ppo --no-probe --no-precision --no-obs --dbs-flips 0 --cpu-sample 0 --no-psnr-check --no-planes --no-scipy"
for r in $(seq 1 $REPS); do
  (cd $OLD && timeout -k 10 300 python bench.py $OLD_Q) > gpurun_out/$T/old_$r.json 2> gpurun_out/$T/old_$r.err || exit 1
  timeout -k 10 300 python bench.py $NEW_Q > gpurun_out/$T/new_$r.json 2> gpurun_out/$T/new_$r.err || exit 1
  for w in old new; do
    python -c "
import json; d = json.loads(open('gpurun_out/$T/${w}_$r.json').read().splitlines()[-1])
print('%-4s %d %9.0f' % ('$w', $r, d['value']), ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in d['passes'].items()))"
  done
done

#!/bin/bash
# Alternated A/B of libhbx builds (same ABI) on the FFT-mode headline only (no side lines):
#   bash tools/ab_libs.sh TAG REPS libhbx libhbx_exp_NAME ...     (run ON the GPU box, repo root)
set -o pipefail
T=$1; REPS=$2; shift 2
L=binary-hologram-reinforcement-learning_amd/hbx
mkdir -p gpurun_out/$T
Q="${AB_Q:---steps 20 --warmup 3 --no-psf --no-ppo --no-probe --no-precision --no-obs --dbs-flips 0 --cpu-sample 0 --no-psnr-check --no-planes --no-crop --no-dropin --no-scipy}"
for r in $(seq 1 $REPS); do
  for lib in "$@"; do
    HBX_LIB=$PWD/$L/$lib.so timeout -k 10 300 python bench.py $Q > gpurun_out/$T/${lib}_$r.json 2> gpurun_out/$T/${lib}_$r.err || exit 1
    python -c "
import json; d = json.loads(open('gpurun_out/$T/${lib}_$r.json').read().splitlines()[-1])
print('%-36s %d %9.0f' % ('$lib', $r, d['value']), ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in d['passes'].items()))"
  done
done

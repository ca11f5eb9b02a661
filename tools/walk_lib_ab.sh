#!/bin/bash
# Device DBS walk A/B of libhbx builds on bench.py's 65,536-candidate 1024x24 prefix
# (run ON the GPU box from the repo root): bash tools/walk_lib_ab.sh TAG libhbx libhbx_exp_X ...
set -o pipefail
T=${1:-wlab}; shift
L=binary-hologram-reinforcement-learning_amd/hbx
mkdir -p gpurun_out/$T
Q="--steps 2 --warmup 1 --no-psf --no-probe --no-precision --no-ppo --no-obs --cpu-sample 0 --no-psnr-check"
i=0
for lib in "$@"; do
  i=$((i + 1))
  HBX_LIB=$PWD/$L/$lib.so timeout -k 10 300 python bench.py $Q > gpurun_out/$T/${i}_$lib.json 2> gpurun_out/$T/${i}_$lib.err || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/$T/${i}_$lib.json').read().splitlines()[-1]); g = d['dbs_greedy']['incremental_mode']
print('%-28s' % '$lib', g['flips_per_s'], g['batches'], g.get('several_images', {}).get('flips_per_s_aggregate'), g['accepted'])"
done

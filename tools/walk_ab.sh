#!/bin/bash
# Persistent vs per-batch fused DBS walk on the bench's 65,536-candidate 1024x24 prefix
# (run ON the GPU box from the repo root): bash tools/walk_ab.sh TAG
set -o pipefail
T=${1:-wab}
mkdir -p gpurun_out/$T
Q="--steps 2 --warmup 1 --no-psf --no-probe --no-precision --no-ppo --no-obs --cpu-sample 0 --no-psnr-check"
for p in 0 1 0 1; do
  HBX_WALK_PERSIST=$p timeout -k 10 300 python bench.py $Q > gpurun_out/$T/p$p.json 2> gpurun_out/$T/p$p.err || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/$T/p$p.json').read().splitlines()[-1]); g = d['dbs_greedy']['incremental_mode']
print('persist $p', g['flips_per_s'], g['batches'], g.get('several_images', {}).get('flips_per_s_aggregate'), g['accepted'])"
done

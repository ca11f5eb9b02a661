#!/bin/bash
# Same-box A/B of the FFT-mode headline and the 256x8 mono line: the round-2 tree (git
# worktree _r02, built in place) against this tree.  Run ON the GPU box from the repo root:
#   bash tools/ab_r02.sh TAG
set -o pipefail
T=${1:-ab_r02}
mkdir -p gpurun_out/$T
Q="--steps 20 --warmup 3 --no-psf --no-probe --no-precision --dbs-flips 0 --cpu-sample 0 --no-psnr-check"
for i in 1 2; do
  (cd _r02 && timeout -k 10 300 python bench.py $Q) > gpurun_out/$T/r02_$i.json 2> gpurun_out/$T/r02_$i.err || exit 1
  timeout -k 10 300 python bench.py $Q --no-obs > gpurun_out/$T/r03_$i.json 2> gpurun_out/$T/r03_$i.err || exit 1
  for v in r02 r03; do
    python -c "
import json; d = json.loads(open('gpurun_out/$T/${v}_$i.json').read().splitlines()[-1])
print('%-6s %9.0f' % ('$v', d['value']), ' '.join('%s %.3f' % (k, v['avg_ms']) for k, v in d['passes'].items()))
m = d['ppo_mono_256']
print('%-6s %9.0f' % ('  256', m['value']), ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in m['passes'].items()))"
  done
done

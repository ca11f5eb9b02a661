#!/bin/bash
# A/B timing of libhbx builds on the FFT-mode headline (csrc: make exp EXP=NAME builds
# hbx/libhbx_exp_NAME.so).  Run ON the GPU box from the repo root:
#   bash tools/ab.sh TAG libhbx libhbx_exp_NAME libhbx libhbx_exp_NAME
set -o pipefail
T=$1; shift
L=binary-hologram-reinforcement-learning_amd/hbx
mkdir -p gpurun_out/$T
Q="--steps 20 --warmup 3 --no-psf --no-ppo --no-probe --no-precision --no-obs --dbs-flips 0 --cpu-sample 0 --no-psnr-check"
i=0
for lib in "$@"; do
  i=$((i + 1))
  HBX_LIB=$PWD/$L/$lib.so timeout -k 10 300 python bench.py $Q > gpurun_out/$T/${i}_${lib}.json 2> gpurun_out/$T/${i}_${lib}.err || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/$T/${i}_${lib}.json').read().splitlines()[-1])
c = d.get('crop_896', {})
print('%-30s %9.0f' % ('$lib', d['value']), ' '.join('%s %.3f' % (k, v['avg_ms']) for k, v in d['passes'].items()),
      '| crop %.0f' % c.get('value', 0), ' '.join('%s %.3f' % (k, v['avg_ms']) for k, v in c.get('passes', {}).items()))"
done

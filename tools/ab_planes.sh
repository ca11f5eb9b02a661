#!/bin/bash
# A/B of libhbx builds on the plane-cached FFT mode (1024x24 and 256x8 mono keys of bench.py).
# Run ON the GPU box from the repo root:  bash tools/ab_planes.sh TAG libhbx libhbx_exp_X ...
set -o pipefail
T=$1; shift
L=binary-hologram-reinforcement-learning_amd/hbx
mkdir -p gpurun_out/$T
Q="--steps 20 --warmup 3 --no-psf --no-probe --no-precision --no-obs --dbs-flips 0 --cpu-sample 0 --no-psnr-check"
i=0
for lib in "$@"; do
  i=$((i + 1))
  HBX_LIB=$PWD/$L/$lib.so timeout -k 10 300 python bench.py $Q > gpurun_out/$T/${i}_${lib}.json 2> gpurun_out/$T/${i}_${lib}.err || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/$T/${i}_${lib}.json').read().splitlines()[-1])
p = d['plane_cached_mode']; m = d['ppo_mono_256']['plane_cached_mode']
print('%-28s fft %8.0f planes %8.0f' % ('$lib', d['value'], p['value']), ' '.join('%s %.3f' % (k, v['avg_ms']) for k, v in p['passes'].items()),
      '| mono fft %8.0f planes %8.0f' % (d['ppo_mono_256']['value'], m['value']), ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in m['passes'].items()))"
done

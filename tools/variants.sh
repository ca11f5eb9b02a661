#!/bin/bash
# Time the FFT-mode passes of several builds of libhbx (timing experiments,
# see csrc/Makefile targets nofft / exp).  Run ON the GPU box from the repo root:
#   bash tools/variants.sh [lib ...]      (default: every hbx/libhbx*.so)
set -o pipefail
LIBDIR=binary-hologram-reinforcement-learning_amd/hbx
LIBS=${*:-$(ls $LIBDIR/libhbx*.so)}
mkdir -p gpurun_out/variants
for lib in $LIBS; do
  name=$(basename $lib .so)
  HBX_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-psf --cpu-sample 0 --dbs-flips 0 --no-probe \
      --no-psnr-check --no-precision --no-ppo > gpurun_out/variants/$name.json 2> gpurun_out/variants/$name.err || exit 1
  python -c "
import json; d = json.load(open('gpurun_out/variants/$name.json'))
print('%-48s %9.0f' % ('$name', d['value']), ' '.join('%s %.3f' % (k, v['avg_ms']) for k, v in d['passes'].items()))"
done

#!/bin/bash
# A/B of the device DBS walk (bench.py's 65,536-candidate prefix) between the default build and
# the four-pixels-per-lane eval kernels (`make exp EXP=PSF_QUAD`).  Run ON the GPU box.
set -o pipefail
L=binary-hologram-reinforcement-learning_amd/hbx
mkdir -p gpurun_out/walkab
for lib in libhbx libhbx_exp_PSF_QUAD libhbx libhbx_exp_PSF_QUAD; do
  HBX_LIB=$PWD/$L/$lib.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-psf --no-ppo --no-probe --cpu-sample 0 --no-psnr-check > gpurun_out/walkab/$lib.json 2> gpurun_out/walkab/$lib.err || exit 1
  python -c "
import json; d = json.load(open('gpurun_out/walkab/$lib.json'))['dbs_greedy']['incremental_mode']
print('%-28s %9.0f candidates/s  %.3f s  accepted %d' % ('$lib', d['flips_per_s'], d['seconds'], d['accepted']))"
done

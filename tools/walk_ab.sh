#!/bin/bash
# A/B of the device DBS walk (bench.py's 65,536-candidate prefix) between builds of libhbx, e.g.
#   bash tools/walk_ab.sh libhbx libhbx_exp_<NAME> libhbx libhbx_exp_<NAME>   (csrc: make exp EXP=<NAME>)
# (profiles/r01_walk_eval_ab.txt came from a one-pixel-per-lane k_walk_eval build, since reverted.)
# Run ON the GPU box.
set -o pipefail
L=binary-hologram-reinforcement-learning_amd/hbx
mkdir -p gpurun_out/walkab
for lib in ${*:-libhbx libhbx}; do
  HBX_LIB=$PWD/$L/$lib.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-psf --no-ppo --no-probe --cpu-sample 0 --no-psnr-check > gpurun_out/walkab/$lib.json 2> gpurun_out/walkab/$lib.err || exit 1
  python -c "
import json; d = json.load(open('gpurun_out/walkab/$lib.json'))['dbs_greedy']['incremental_mode']
print('%-28s %9.0f candidates/s  %.3f s  accepted %d' % ('$lib', d['flips_per_s'], d['seconds'], d['accepted']))"
done

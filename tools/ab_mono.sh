#!/bin/bash
# A/B of libhbx builds on the 256x256x8 mono step (tools/pg_overhead.py, sampled pass timing).
# Run ON the GPU box from the repo root:  bash tools/ab_mono.sh libhbx libhbx_exp_NAME ...
set -o pipefail
L=binary-hologram-reinforcement-learning_amd/hbx
for lib in "$@"; do
  echo -n "$lib: "
  HBX_LIB=$PWD/$L/$lib.so timeout -k 10 200 python tools/pg_overhead.py none 0 4 2>/dev/null | grep rep3 || exit 1
done

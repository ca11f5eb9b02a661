#!/bin/bash
# FFT-mode device walk (hbx_dbs_walk_planes) A/B of libhbx builds on tools/dbs_walk_bench.py's
# 16,384-candidate 1024x24 prefix.  Run ON the GPU box from the repo root:
#   bash tools/fftwalk_lib_ab.sh libhbx libhbx_exp_X ...
set -o pipefail
L=binary-hologram-reinforcement-learning_amd/hbx
for lib in "$@"; do
  echo -n "$lib: "
  HBX_LIB=$PWD/$L/$lib.so timeout -k 10 200 python tools/dbs_walk_bench.py --trace 2>/dev/null | grep device_walk || exit 1
done

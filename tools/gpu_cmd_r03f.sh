#!/bin/bash
# r03f: plane-cache step-by-step debug, then which bf16 pass is non-deterministic at N = 1024.
set -o pipefail
mkdir -p gpurun_out/r03f
L=binary-hologram-reinforcement-learning_amd/hbx
timeout -k 10 300 python -u tools/planes_debug.py > gpurun_out/r03f/planes_debug.txt 2>&1
rc=$?; tail -30 gpurun_out/r03f/planes_debug.txt
if [ $rc -gt 1 ]; then exit $rc; fi
for lib in libhbx libhbx_exp_SK_COL_ONLY libhbx_exp_SK_ROWFWD_ONLY; do
  echo "== $lib"
  HBX_LIB=$PWD/$L/$lib.so timeout -k 10 200 python -u tools/bf16_diag.py det 2>&1 | grep -v amdgpu.ids || exit 1
done

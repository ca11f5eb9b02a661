#!/bin/bash
# r03g: plane-cache debug + tests (two spares), bf16 determinism with the rounding moved to the
# staging write, then the whole -m gpu suite + bench line.
set -o pipefail
mkdir -p gpurun_out/r03g
L=binary-hologram-reinforcement-learning_amd/hbx
timeout -k 10 300 python -u tools/planes_debug.py > gpurun_out/r03g/planes_debug.txt 2>&1
rc=$?; grep -c differing gpurun_out/r03g/planes_debug.txt; grep "reward equal False" gpurun_out/r03g/planes_debug.txt | head -3
if [ $rc -gt 1 ]; then exit $rc; fi
for lib in libhbx libhbx_exp_SK_COL_ONLY; do
  echo "== $lib"
  HBX_LIB=$PWD/$L/$lib.so timeout -k 10 200 python -u tools/bf16_diag.py det 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_planes.py -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03g/planes_tests.txt 2>&1
rc=$?; tail -8 gpurun_out/r03g/planes_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_round.sh r03g

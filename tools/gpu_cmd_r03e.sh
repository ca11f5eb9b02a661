#!/bin/bash
# r03e GPU call: plane-cached mode tests first (new kernels), bf16 determinism diagnostic, then
# the whole -m gpu suite + bench line.  Stops at the first fault / timeout.
set -o pipefail
mkdir -p gpurun_out/r03e
timeout -k 10 400 python -u -m pytest tests/test_gpu_planes.py -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03e/planes_tests.txt 2>&1
rc=$?; tail -8 gpurun_out/r03e/planes_tests.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/bf16_diag.py > gpurun_out/r03e/bf16.txt 2>&1
rc2=$?; tail -14 gpurun_out/r03e/bf16.txt
if [ $rc2 -gt 1 ]; then exit $rc2; fi
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_round.sh r03e

#!/bin/bash
# r03d GPU call: bf16 per-flip diagnostic, the -m gpu suite + bench line on HEAD, then the
# walk dedup A/B and its walk tests.  Stops at the first fault / timeout.
set -o pipefail
mkdir -p gpurun_out/r03d
timeout -k 10 300 python -u tools/bf16_diag.py > gpurun_out/r03d/bf16.txt 2>&1
rc=$?; tail -12 gpurun_out/r03d/bf16.txt
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpu_round.sh r03d
rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/walk_lib_ab.sh r03d_wab libhbx libhbx_exp_WALK_DEDUP libhbx libhbx_exp_WALK_DEDUP || exit 1
HBX_LIB=$PWD/binary-hologram-reinforcement-learning_amd/hbx/libhbx_exp_WALK_DEDUP.so timeout -k 10 400 \
  python -u -m pytest tests -m gpu -k "walk or greedy" -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03d/dedup_tests.txt 2>&1
tail -3 gpurun_out/r03d/dedup_tests.txt

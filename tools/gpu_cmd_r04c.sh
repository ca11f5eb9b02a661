#!/bin/bash
# r04c: the whole -m gpu suite + the default bench line on main (plane-cached device-walk greedy,
# fused recon reconcile, 896 tiles), then tools/obs_cost.py at 256 and 1024 (SB3-facing step
# overhead decomposition).
set -o pipefail
bash tools/gpu_round.sh r04c
rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/obs_cost.py 256 > gpurun_out/r04c/obs_cost_256.txt 2>&1 || exit 21
timeout -k 10 300 python tools/obs_cost.py 1024 > gpurun_out/r04c/obs_cost_1024.txt 2>&1 || exit 22
cat gpurun_out/r04c/obs_cost_*.txt | grep "N="
exit $rc

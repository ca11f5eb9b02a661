#!/bin/bash
# r03l: the whole -m gpu suite + full bench line on HEAD after the container re-creation, then the
# rocprofv3 set (kernel trace + FETCH/WRITE/SQ/LDS passes) of the same code, summarised on the box
# (the raw per-dispatch CSVs are dropped: they exceed gpurun's 64-MiB copy-back).
set -o pipefail
bash tools/gpu_round.sh r03l
rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/profile.sh r03l > /dev/null || exit 10
python3 tools/pmc_summary.py gpurun_out/prof_r03l --jobs 128 --N 1024 --out gpurun_out/prof_r03l/pmc_summary.json \
  > gpurun_out/prof_r03l/pmc_summary.txt 2>&1 || exit 11
find gpurun_out/prof_r03l \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
tail -30 gpurun_out/prof_r03l/pmc_summary.txt
exit $rc

#!/bin/bash
# r03h: rocprofv3 kernel trace + PMC passes on HEAD (headline 1024x24 and 256x8 mono).  The
# summaries are made ON the box and the raw per-dispatch CSVs dropped, so gpurun_out/ stays far
# below gpurun's 64 MiB copy-back limit.
set -o pipefail
bash tools/profile.sh r03h > /dev/null || exit $?
bash tools/prof_mono.sh r03h > /dev/null || exit $?
python3 tools/pmc_summary.py gpurun_out/prof_r03h --jobs 128 --N 1024 --out gpurun_out/prof_r03h/pmc_summary.json \
  > gpurun_out/prof_r03h/pmc_summary.txt 2>&1 || exit 7
python3 tools/pmc_summary.py gpurun_out/prof_mono_r03h --jobs 128 --N 256 --out gpurun_out/prof_mono_r03h/pmc_summary.json \
  > gpurun_out/prof_mono_r03h/pmc_summary.txt 2>&1 || exit 8
find gpurun_out/prof_r03h gpurun_out/prof_mono_r03h \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \
  -o -name "*.db" \) -delete
tail -30 gpurun_out/prof_r03h/pmc_summary.txt
du -sh gpurun_out
bash tools/ab_planes.sh r03h_planes libhbx libhbx_exp_PLANES_TWO_SETS libhbx_exp_PLANES_TWO_SETS_PLANES_C2 libhbx libhbx_exp_PLANES_TWO_SETS libhbx_exp_PLANES_TWO_SETS_PLANES_C2

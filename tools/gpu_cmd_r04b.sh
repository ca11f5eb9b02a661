#!/bin/bash
# r04b: rocprofv3 sets (kernel trace + FETCH / WRITE / SQ / LDS passes) of the r04 code at
# N = 1024 (k_col2 stage regions) and at the 896 crop (k_rowfwd896 / k_col896 rewrite),
# summarised on the box; raw per-dispatch CSVs dropped (64-MiB copy-back).
set -o pipefail
bash tools/profile.sh r04b > /dev/null || exit 10
python3 tools/pmc_summary.py gpurun_out/prof_r04b --jobs 128 --N 1024 --out gpurun_out/prof_r04b/pmc_summary.json \
  > gpurun_out/prof_r04b/pmc_summary.txt 2>&1 || exit 11
find gpurun_out/prof_r04b \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
bash tools/profile.sh r04b_896 --size 896 --no-ppo > /dev/null || exit 12
python3 tools/pmc_summary.py gpurun_out/prof_r04b_896 --jobs 128 --N 896 \
  --out gpurun_out/prof_r04b_896/pmc_summary.json > gpurun_out/prof_r04b_896/pmc_summary.txt 2>&1 || exit 13
find gpurun_out/prof_r04b_896 \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
python3 - <<'PY'
import json
for t in ("r04b", "r04b_896"):
    d = json.load(open(f"gpurun_out/prof_{t}/pmc_summary.json"))
    for k, v in d["kernels"].items():
        print(t, k, round(v["avg_ms"], 4), "alg", round(v["alg_GBs"] or 0), "hbm x",
              round((v["hbm_bytes_per_launch"] or 0) / (v["alg_bytes_per_launch"] or 1), 3),
              "bank", v.get("SQ_LDS_BANK_CONFLICT"), "vgpr", v.get("vgpr"))
PY

#!/bin/bash
# r04h: r04g (obs tests, SB3 step host phases, obs_cost, k_rowfwd896 A/B), then the default
# bench line and the rocprofv3 sets (trace + FETCH / WRITE / SQ / LDS) at 1024 and the 896 crop.
set -o pipefail
bash tools/gpu_cmd_r04g.sh || exit $?
T=gpurun_out/r04h
mkdir -p $T
timeout -k 10 600 python bench.py > $T/bench.json 2> $T/bench.err || { tail -20 $T/bench.err; exit 30; }
python3 -c "
import json; d = json.loads(open('$T/bench.json').read().splitlines()[-1])
print('headline', d['value'], d['roofline']['frac'], {k: v['avg_ms'] for k, v in d['passes'].items()})
print('dbs', d.get('dbs_greedy', {}).get('flips_per_s'), 'crop', d.get('crop_896', {}).get('value'))
m = d.get('ppo_mono_256', {}); print('mono', m.get('value'), 'obs', m.get('vecenv_step_obs', {}).get('obs_overhead_frac'))"
bash tools/profile.sh r04h > /dev/null || exit 31
python3 tools/pmc_summary.py gpurun_out/prof_r04h --jobs 128 --N 1024 --out gpurun_out/prof_r04h/pmc_summary.json \
  > gpurun_out/prof_r04h/pmc_summary.txt 2>&1 || exit 32
find gpurun_out/prof_r04h \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
bash tools/profile.sh r04h_896 --size 896 --no-ppo > /dev/null || exit 33
python3 tools/pmc_summary.py gpurun_out/prof_r04h_896 --jobs 128 --N 896 \
  --out gpurun_out/prof_r04h_896/pmc_summary.json > gpurun_out/prof_r04h_896/pmc_summary.txt 2>&1 || exit 34
find gpurun_out/prof_r04h_896 \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
python3 - <<'PY'
import json
for t in ("r04h", "r04h_896"):
    d = json.load(open(f"gpurun_out/prof_{t}/pmc_summary.json"))
    for k, v in d["kernels"].items():
        print(t, k, round(v["avg_ms"], 4), "alg", round(v["alg_GBs"] or 0), "hbm x",
              round((v["hbm_bytes_per_launch"] or 0) / (v["alg_bytes_per_launch"] or 1), 3),
              "bank", v.get("SQ_LDS_BANK_CONFLICT"), "vgpr", v.get("vgpr"))
PY

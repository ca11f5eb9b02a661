#!/bin/bash
# r04m: the round-end checks on the current tree -- GPU suite, smoke(), default bench line -- and
# the 896 rocprofv3 set after k_rowfwd896's 8 row blocks per workgroup
set -o pipefail
T=gpurun_out/r04m
mkdir -p $T
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > $T/gpu_tests.log 2>&1 || { tail -30 $T/gpu_tests.log; exit 19; }
tail -2 $T/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $T/smoke.log 2>&1 || { tail -20 $T/smoke.log; exit 20; }
tail -1 $T/smoke.log
timeout -k 10 600 python bench.py > $T/bench.json 2> $T/bench.err || { tail -20 $T/bench.err; exit 30; }
python3 -c "
import json; d = json.loads(open('$T/bench.json').read().splitlines()[-1])
print('headline', d['value'], d['roofline']['frac'], {k: v['avg_ms'] for k, v in d['passes'].items()})
print('dbs', d.get('dbs_greedy', {}).get('flips_per_s'), 'crop', d.get('crop_896', {}).get('value'), {k: v['avg_ms'] for k, v in d.get('crop_896', {}).get('passes', {}).items()})
m = d.get('ppo_mono_256', {}); v = m.get('vecenv_step_obs', {}); print('mono', m.get('value'), 'obs', v.get('obs_overhead_frac'), v.get('overhead_vs_pure_device_step'), v.get('ms_per_step'), v.get('pure_device_step_ms'))
v = d.get('vecenv_step_obs', {}); print('1024 obs', v.get('obs_overhead_frac'), v.get('overhead_vs_pure_device_step'))"
bash tools/profile.sh r04m_896 --size 896 --no-ppo > /dev/null || exit 33
python3 tools/pmc_summary.py gpurun_out/prof_r04m_896 --jobs 128 --N 896 \
  --out gpurun_out/prof_r04m_896/pmc_summary.json > gpurun_out/prof_r04m_896/pmc_summary.txt 2>&1 || exit 34
find gpurun_out/prof_r04m_896 \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/prof_r04m_896/pmc_summary.json"))
for k, v in d["kernels"].items():
    print("r04m_896", k, round(v["avg_ms"], 4), "alg", round(v["alg_GBs"] or 0), "hbm x",
          round((v["hbm_bytes_per_launch"] or 0) / (v["alg_bytes_per_launch"] or 1), 3),
          "bank", v.get("SQ_LDS_BANK_CONFLICT"), "vgpr", v.get("vgpr"))
PY

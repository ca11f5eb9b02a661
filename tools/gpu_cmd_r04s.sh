#!/bin/bash
# r04s: final GPU suite + smoke + default bench line on the final tree
set -o pipefail
T=gpurun_out/r04s
mkdir -p $T
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $T/gpu_tests.log 2>&1 || { tail -30 $T/gpu_tests.log; exit 19; }
tail -2 $T/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $T/smoke.log 2>&1 || { tail -20 $T/smoke.log; exit 20; }
tail -1 $T/smoke.log
timeout -k 10 600 python bench.py > $T/bench.json 2> $T/bench.err || { tail -20 $T/bench.err; exit 30; }
python3 -c "
import json; d = json.loads(open('$T/bench.json').read().splitlines()[-1])
print('headline', d['value'], d['roofline']['frac'], {k: v['avg_ms'] for k, v in d['passes'].items()})
g = d.get('dbs_greedy', {}); print('dbs', g.get('flips_per_s'), 'many', g.get('several_images', {}).get('flips_per_s_aggregate'), 'crop', d.get('crop_896', {}).get('value'))
m = d.get('ppo_mono_256', {}); v = m.get('vecenv_step_obs', {}); print('mono', m.get('value'), 'obs', v.get('obs_overhead_frac'), v.get('overhead_vs_pure_device_step'))"

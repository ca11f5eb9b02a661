#!/bin/bash
# r04o: final-state checks -- GPU suite, smoke(), the C-ABI host program, the default bench line,
# and the world-2 self-launch rehearsal
set -o pipefail
T=gpurun_out/r04o
mkdir -p $T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $T/gpu_tests.log 2>&1 || { tail -30 $T/gpu_tests.log; exit 19; }
tail -2 $T/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $T/smoke.log 2>&1 || { tail -20 $T/smoke.log; exit 20; }
tail -1 $T/smoke.log
timeout -k 10 100 ./binary-hologram-reinforcement-learning_amd/hbx/env_step_host 128 300 > $T/c_host.txt 2>&1 || { cat $T/c_host.txt; exit 21; }
cat $T/c_host.txt
timeout -k 10 600 python bench.py > $T/bench.json 2> $T/bench.err || { tail -20 $T/bench.err; exit 30; }
python3 -c "
import json; d = json.loads(open('$T/bench.json').read().splitlines()[-1])
print('headline', d['value'], d['roofline']['frac'], {k: v['avg_ms'] for k, v in d['passes'].items()})
print('dbs', d.get('dbs_greedy', {}).get('flips_per_s'), 'crop', d.get('crop_896', {}).get('value'))
m = d.get('ppo_mono_256', {}); v = m.get('vecenv_step_obs', {}); print('mono', m.get('value'), 'obs', v.get('obs_overhead_frac'), v.get('overhead_vs_pure_device_step'))"
HBX_BENCH_REHEARSE_ONE_GPU=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 2 > $T/rehearse_world2.json 2> $T/rehearse_world2.log || { tail -20 $T/rehearse_world2.log; exit 24; }
python3 -c "import json; d = json.loads(open('$T/rehearse_world2.json').read().splitlines()[-1]); print('world2', d['n_gpus'], d['value'], d['ranks_seen'])"

#!/bin/bash
# r04p: the pipelined cached-plane reads of k_rowinv_d's plane-cached step -- the plane / walk
# tests (bit-exact to the FFT mode), the walk, the planes-mode bench lines
set -o pipefail
T=gpurun_out/r04p
mkdir -p $T
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_planes.py tests/test_gpu_dbs_headline.py tests/test_gpu_obs.py -m gpu > $T/tests.log 2>&1 || { tail -30 $T/tests.log; exit 19; }
tail -2 $T/tests.log
timeout -k 10 200 python tools/dbs_walk_bench.py --flips 65536 --trace > $T/walk.txt 2>&1 || { tail $T/walk.txt; exit 20; }
grep device_walk $T/walk.txt
timeout -k 10 600 python bench.py > $T/bench.json 2> $T/bench.err || { tail -20 $T/bench.err; exit 30; }
python3 -c "
import json; d = json.loads(open('$T/bench.json').read().splitlines()[-1])
print('headline', d['value'], {k: v['avg_ms'] for k, v in d['passes'].items()})
p = d['plane_cached_mode']; print('planes', p['value'], {k: (v['avg_ms'], round(v['achieved_GBs'] / 8000, 3)) for k, v in p['passes'].items()})
m = d['ppo_mono_256']; p = m.get('plane_cached_mode', {}); print('mono', m['value'], 'planes', p.get('value'), {k: v['avg_ms'] for k, v in p.get('passes', {}).items()})
print('dbs', d.get('dbs_greedy', {}).get('flips_per_s'))"

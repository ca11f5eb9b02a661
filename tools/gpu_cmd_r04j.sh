#!/bin/bash
# r04j: GPU suite (k_rowfwd896 at 8 row blocks, blocking readback), the walk at k_max 256 after
# the one-pass K choice, host phases, and the default bench line
set -o pipefail
T=gpurun_out/r04j
mkdir -p $T
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $T/gpu_tests.log 2>&1 || { tail -30 $T/gpu_tests.log; exit 19; }
tail -2 $T/gpu_tests.log
timeout -k 10 200 python tools/dbs_walk_bench.py --flips 65536 --trace > $T/walk.txt 2>&1 || { tail $T/walk.txt; exit 20; }
grep device_walk $T/walk.txt
timeout -k 10 200 python tools/step_host.py > $T/step_host.txt 2>&1 || { cat $T/step_host.txt; exit 21; }
grep -v amdgpu $T/step_host.txt
timeout -k 10 600 python bench.py > $T/bench.json 2> $T/bench.err || { tail -20 $T/bench.err; exit 30; }
python3 -c "
import json; d = json.loads(open('$T/bench.json').read().splitlines()[-1])
print('headline', d['value'], d['roofline']['frac'], {k: v['avg_ms'] for k, v in d['passes'].items()})
print('dbs', d.get('dbs_greedy', {}).get('flips_per_s'), 'crop', d.get('crop_896', {}).get('value'), {k: v['avg_ms'] for k, v in d.get('crop_896', {}).get('passes', {}).items()})
m = d.get('ppo_mono_256', {}); print('mono', m.get('value'), 'obs', m.get('vecenv_step_obs', {}).get('obs_overhead_frac'))"
# per-kernel durations of the adaptive FFT-mode walk (16,384 candidates)
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $T/walk_trace -o run -- python3 tools/dbs_walk_bench.py --flips 16384 --trace > $T/walk_trace.log 2>&1 || exit 31
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r04j/walk_trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("%-60s %8s %10.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
python3 tools/step_gap.py --gaps gpurun_out/r04j/walk_trace > $T/walk_gaps.txt 2>&1; head -12 $T/walk_gaps.txt
find $T/walk_trace -name "*trace.csv" -delete

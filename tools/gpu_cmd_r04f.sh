#!/bin/bash
# r04f: the whole GPU suite after fusing the row-block reduction into the env-step finalize and
# the walk; the SB3 step cost at 256 / 1024 (tools/obs_cost.py) and its timeline.
set -o pipefail
T=gpurun_out/r04f
mkdir -p $T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $T/gpu_tests.log 2>&1 || { tail -30 $T/gpu_tests.log; exit 19; }
tail -2 $T/gpu_tests.log
timeout -k 10 200 python tools/obs_cost.py 256 > $T/obs_cost.txt 2>&1 || exit 20
timeout -k 10 200 python tools/obs_cost.py 1024 >> $T/obs_cost.txt 2>&1 || exit 21
grep -v amdgpu.ids $T/obs_cost.txt
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $T/step_trace -o run -- python3 tools/step_gap.py --steps 200 > $T/step_trace.log 2>&1 || exit 22
python3 tools/step_gap.py --summarize $T/step_trace > $T/step_gaps.txt 2>&1
python3 tools/step_gap.py --gaps $T/step_trace >> $T/step_gaps.txt 2>&1
cat $T/step_gaps.txt
find $T/step_trace -name "*.csv" -delete
for k in 2 4 6; do
  timeout -k 10 200 python tools/dbs_walk_bench.py --flips 16384 --k $k >> $T/dbs_walk_k.txt 2>&1 || exit 23
done
grep device_walk $T/dbs_walk_k.txt
# bench.py --gpus 2 with no outer launcher starts its own two ranks
HBX_BENCH_REHEARSE_ONE_GPU=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 2 > $T/rehearse_world2.json 2> $T/rehearse_world2.log || { tail -20 $T/rehearse_world2.log; exit 24; }
cat $T/rehearse_world2.json

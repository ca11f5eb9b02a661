#!/bin/bash
# r04e: GPU timelines -- the device-decided DBS walk (K = 4 and adaptive) and the SB3-facing mono
# step -- for the kernel-boundary gaps (tools/step_gap.py), plus dbs_walk_bench at fixed K.
set -o pipefail
T=gpurun_out/r04e
mkdir -p $T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_planes.py tests/test_gpu_dbs_headline.py -m gpu > $T/walk_tests.log 2>&1 || { tail -30 $T/walk_tests.log; exit 19; }
tail -2 $T/walk_tests.log
for k in 4 8; do
  timeout -k 10 200 python tools/dbs_walk_bench.py --flips 16384 --trace --k $k >> $T/dbs_walk_k.txt 2>&1 || exit 20
done
cat $T/dbs_walk_k.txt | grep device_walk
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $T/walk_trace -o run -- python3 tools/dbs_walk_bench.py --flips 4096 --trace --k 4 > $T/walk_trace.log 2>&1 || exit 21
python3 tools/step_gap.py --gaps $T/walk_trace > $T/walk_gaps.txt 2>&1
cat $T/walk_gaps.txt
find $T/walk_trace -name "*.csv" -delete
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $T/step_trace -o run -- python3 tools/step_gap.py --steps 200 > $T/step_trace.log 2>&1 || exit 22
python3 tools/step_gap.py --summarize $T/step_trace > $T/step_gaps.txt 2>&1
python3 tools/step_gap.py --gaps $T/step_trace >> $T/step_gaps.txt 2>&1
cat $T/step_gaps.txt
find $T/step_trace -name "*.csv" -delete
timeout -k 10 300 python tools/obs_cost.py > $T/obs_cost.txt 2>&1 || exit 23
cat $T/obs_cost.txt

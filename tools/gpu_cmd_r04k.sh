#!/bin/bash
# r04k: the LDS-prefetching k_walk_planes -- walk tests, 65,536-candidate walk, kernel durations
set -o pipefail
T=gpurun_out/r04k
mkdir -p $T
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_dbs_headline.py -m gpu -k "plane_cache or ratio05 or fft_greedy" > $T/walk_tests.log 2>&1 || { tail -30 $T/walk_tests.log; exit 19; }
tail -2 $T/walk_tests.log
timeout -k 10 200 python tools/dbs_walk_bench.py --flips 65536 --trace > $T/walk.txt 2>&1 || { tail $T/walk.txt; exit 20; }
grep device_walk $T/walk.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $T/walk_trace -o run -- python3 tools/dbs_walk_bench.py --flips 16384 --trace > $T/walk_trace.log 2>&1 || exit 31
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r04k/walk_trace/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:5]:
        print("%-60s %8s %10.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
find $T/walk_trace -name "*trace.csv" -delete

#!/bin/bash
# r04i: why the bench's adaptive FFT-mode walk ran 253 us per batch (r04h) against 87 us at K = 4
# in dbs_walk_bench (r04f): same tool, 65,536 candidates, k_max 256 (adaptive) vs 3 / 4
set -o pipefail
T=gpurun_out/r04i
mkdir -p $T
for k in 0 3 4; do
  timeout -k 10 200 python tools/dbs_walk_bench.py --flips 65536 --trace --k $k >> $T/walk.txt 2>&1 || { tail $T/walk.txt; exit 20; }
done
grep device_walk $T/walk.txt

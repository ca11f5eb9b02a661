#!/bin/bash
# r03p: the 4-image full DBS_1024_24 sweep (4 x 25,165,824 candidates, walks side by side) on r03 code
set -o pipefail
mkdir -p gpurun_out/r03p
timeout -k 10 1050 python -u tools/dbs_full_sweep_many.py 4 > gpurun_out/r03p/dbs_full_sweep_4images.txt 2>&1
rc=$?
tail -2 gpurun_out/r03p/dbs_full_sweep_4images.txt
exit $rc

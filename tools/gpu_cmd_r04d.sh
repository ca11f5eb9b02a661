#!/bin/bash
# r04d: the DBS tests (plane cache / device walk with up to G accepts per batch vs the full
# re-propagation, the oracle fixtures), tools/dbs_walk_bench.py, and a kernel trace of the walk.
set -o pipefail
T=gpurun_out/r04d
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_gpu_dbs_headline.py -m gpu -v --timeout 300 --timeout-method thread \
  > $T/gpu_tests_dbs.txt 2>&1
rc=$?
tail -3 $T/gpu_tests_dbs.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/dbs_walk_bench.py --flips 16384 > $T/dbs_walk_bench.txt 2>&1 || exit 21
cat $T/dbs_walk_bench.txt
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $T/walk_trace -o run -- python3 tools/dbs_walk_bench.py --flips 4096 --trace > $T/walk_trace.log 2>&1 || exit 22
find $T/walk_trace -name "*kernel_trace.csv" -delete
head -20 $T/walk_trace/run_kernel_stats.csv | cut -c1-160
exit $rc

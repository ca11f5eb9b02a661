#!/bin/bash
# r03j: graph-replayed step tests, the whole -m gpu suite + full bench line, the 896 crop line and
# the full 25.2 M-candidate DBS_1024_24 sweep on the r03 code.
set -o pipefail
mkdir -p gpurun_out/r03j
timeout -k 10 300 python -u -m pytest tests/test_gpu_obs.py -v -k graph --timeout 200 --timeout-method thread \
  > gpurun_out/r03j/graph_tests.txt 2>&1
rc=$?; tail -4 gpurun_out/r03j/graph_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_round.sh r03j
rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --size 896 --steps 20 --no-psf --no-ppo --no-probe --no-precision --no-obs \
  --dbs-flips 0 --cpu-sample 0 --no-planes > gpurun_out/r03j/bench_896.json 2> gpurun_out/r03j/bench_896.err || exit 3
python -c "import json; d=json.loads(open('gpurun_out/r03j/bench_896.json').read().splitlines()[-1]); print('896', d['value'], d['ms_per_step'])"
timeout -k 10 420 python -u tools/dbs_full_sweep.py > gpurun_out/r03j/dbs_full_sweep.txt 2>&1
tail -2 gpurun_out/r03j/dbs_full_sweep.txt

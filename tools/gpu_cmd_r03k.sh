#!/bin/bash
# r03k: default bench wall time (the driver's N = 1 call) and the world-2 bench path rehearsed on
# one GPU (gloo, both ranks on cuda:0: a code-path check, not a scaling measurement)
set -o pipefail
mkdir -p gpurun_out/r03k
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03k/smoke.txt 2>&1 || exit 4
tail -1 gpurun_out/r03k/smoke.txt
s=$(date +%s.%N)
timeout -k 10 600 python bench.py > gpurun_out/r03k/bench_default.json 2> gpurun_out/r03k/bench_default.err || exit 1
e=$(date +%s.%N)
python -c "print('default bench wall s', round($e - $s, 1))" | tee gpurun_out/r03k/bench_default_wall.txt
HBX_BENCH_REHEARSE_ONE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 \
  > gpurun_out/r03k/rehearse_world2.json 2> gpurun_out/r03k/rehearse_world2.err || exit 2
python -c "
import json; d=json.loads(open('gpurun_out/r03k/rehearse_world2.json').read().splitlines()[-1])
print('world2', d['n_gpus'], d['value'], d['ranks_seen'], 'planes' in str(d.keys()), d.get('plane_cached_mode', {}).get('value'))"

#!/bin/bash
# r04a: the -m gpu suite + bench line on the r04 k_col2 (conflict-free stage regions, soffset-0
# stage stores); then the ITER = 1 k_col2<16> exp build (the r03 anomaly) through the flip-map
# test and a mono 256 timing; then the world-2 rehearsal of bench.py's self-launched ranks.
set -o pipefail
bash tools/gpu_round.sh r04a
rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
T=gpurun_out/r04a
HBX_LIB=$PWD/binary-hologram-reinforcement-learning_amd/hbx/libhbx_exp_COL2_ITER1.so timeout -k 10 300 \
  python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_planes.py tests/test_gpu_obs.py -m gpu -v \
  -k "256 or mono or every_flip" --timeout 200 --timeout-method thread > $T/iter1_tests.txt 2>&1
irc=$?
tail -3 $T/iter1_tests.txt
if [ $irc -gt 1 ]; then exit $irc; fi
for lib in libhbx.so libhbx_exp_COL2_ITER1.so libhbx.so libhbx_exp_COL2_ITER1.so; do
  HBX_LIB=$PWD/binary-hologram-reinforcement-learning_amd/hbx/$lib timeout -k 10 200 python bench.py --steps 20 \
    --warmup 3 --cpu-sample 0 --dbs-flips 0 --no-probe --no-precision --no-obs --no-psf --no-planes \
    --no-psnr-check --no-scipy > $T/mono_$lib.json 2>> $T/mono.err || exit 20
  python3 -c "import json,sys; d=json.load(open('$T/mono_$lib.json')); m=d['ppo_mono_256']; print('$lib', d['value'], d['passes']['k_col']['avg_ms'], m['ms_per_step'], {k: v['avg_ms'] for k, v in m['passes'].items()})" | tee -a $T/iter1_ab.txt
done
HBX_BENCH_REHEARSE_ONE_GPU=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 10 --warmup 2 --cpu-sample 0 \
  --no-psf --no-planes --no-ppo > $T/rehearse_world2.json 2> $T/rehearse_world2.err
wrc=$?
tail -c 1500 $T/rehearse_world2.json
echo "rehearse rc=$wrc"
exit $(( rc > wrc ? rc : wrc ))

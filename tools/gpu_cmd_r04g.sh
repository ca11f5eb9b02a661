#!/bin/bash
# r04g: the SB3 step after the host-mapped readback, first-pass action decode and the settle
# copy behind the readback: obs tests, host phases, obs_cost 256 / 1024
set -o pipefail
T=gpurun_out/r04g
mkdir -p $T
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_obs.py tests/test_gpu_planes.py -m gpu > $T/obs_tests.log 2>&1 || { tail -30 $T/obs_tests.log; exit 19; }
tail -2 $T/obs_tests.log
timeout -k 10 200 python tools/step_host.py > $T/step_host.txt 2>&1 || { cat $T/step_host.txt; exit 20; }
cat $T/step_host.txt
timeout -k 10 200 python tools/obs_cost.py 256 > $T/obs_cost.txt 2>&1 || exit 21
timeout -k 10 200 python tools/obs_cost.py 1024 >> $T/obs_cost.txt 2>&1 || exit 22
grep -v amdgpu.ids $T/obs_cost.txt
# k_rowfwd896 row blocks per workgroup (k_rowfwd896 >= 0.6 of 8 TB/s)
bash tools/ab.sh r04g_ab libhbx libhbx_exp_RIT896_2 libhbx_exp_RIT896_7 libhbx_exp_RIT896_8 libhbx || exit 23

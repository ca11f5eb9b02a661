#!/bin/bash
# r03m: k_rowinv_d at three workgroups per CU (EXP ROWINV3: split re/im FFT tile, 42 KB LDS) --
# bitwise A/B of the propagation against the product build, then headline and mono timing A/B.
set -o pipefail
L=$PWD/binary-hologram-reinforcement-learning_amd/hbx
mkdir -p gpurun_out/r03m
HBX_LIB=$L/libhbx.so timeout -k 10 200 python tools/lib_bitcmp.py dump gpurun_out/r03m/a.npz || exit 1
HBX_LIB=$L/libhbx_exp_ROWINV3.so timeout -k 10 200 python tools/lib_bitcmp.py dump gpurun_out/r03m/b.npz || exit 2
python tools/lib_bitcmp.py cmp gpurun_out/r03m/a.npz gpurun_out/r03m/b.npz | tee gpurun_out/r03m/bitcmp.txt
rm -f gpurun_out/r03m/*.npz
bash tools/ab.sh r03m_ab libhbx libhbx_exp_ROWINV3 libhbx libhbx_exp_ROWINV3 | tee gpurun_out/r03m/ab.txt || exit 3
bash tools/ab_mono.sh libhbx libhbx_exp_ROWINV3 libhbx libhbx_exp_ROWINV3 | tee gpurun_out/r03m/ab_mono.txt || exit 4

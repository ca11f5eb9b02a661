set -o pipefail
mkdir -p gpurun_out/r02_rf
Q="--steps 20 --no-psf --no-ppo --no-probe --no-scipy --no-precision --cpu-sample 1 --dbs-flips 4096"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r02_rf/parity.txt 2>&1 &&
timeout -k 10 200 python bench.py $Q > gpurun_out/r02_rf/new.json 2> gpurun_out/r02_rf/new.err &&
HBX_LIB=$PWD/binary-hologram-reinforcement-learning_amd/hbx/libhbx_exp_ROWFWD_WIDE.so timeout -k 10 200 python bench.py $Q > gpurun_out/r02_rf/wide.json 2> gpurun_out/r02_rf/wide.err &&
timeout -k 10 200 python bench.py $Q > gpurun_out/r02_rf/new2.json 2>> gpurun_out/r02_rf/new.err

# A/B timing of pass variants (exp libraries built in-tree by `make exp EXP=...`)
set -o pipefail
mkdir -p gpurun_out/r02_rf
Q="--steps 20 --no-psf --no-ppo --no-probe --no-scipy --no-precision --cpu-sample 1 --dbs-flips 4096"
L=$PWD/binary-hologram-reinforcement-learning_amd/hbx
timeout -k 10 200 python bench.py $Q > gpurun_out/r02_rf/new.json 2> gpurun_out/r02_rf/new.err &&
for v in ${VARIANTS}; do
  HBX_LIB=$L/libhbx_exp_$v.so timeout -k 10 200 python bench.py $Q > gpurun_out/r02_rf/$v.json 2> gpurun_out/r02_rf/$v.err || exit 1
done &&
timeout -k 10 200 python bench.py $Q > gpurun_out/r02_rf/new2.json 2>> gpurun_out/r02_rf/new.err

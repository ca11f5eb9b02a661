set -o pipefail
L=binary-hologram-reinforcement-learning_amd/hbx
mkdir -p gpurun_out/psfab
for lib in ${*:-libhbx libhbx_exp_PSF_QUAD libhbx libhbx_exp_PSF_QUAD}; do
  HBX_LIB=$PWD/$L/$lib.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --psf-steps 300 --cpu-sample 0 --dbs-flips 0 --no-probe --no-psnr-check --no-ppo > gpurun_out/psfab/$lib.json 2> gpurun_out/psfab/$lib.err || exit 1
  python -c "
import json; d = json.load(open('gpurun_out/psfab/$lib.json'))['incremental_psf_mode']
print('%-28s %9.0f' % ('$lib', d['value']), ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in d['passes'].items()))"
done

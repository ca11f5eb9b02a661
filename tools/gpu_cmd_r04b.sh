#!/bin/bash
# r04b: GPU tests of the r04 896 passes (B slot tiles, direct-load k_rowinv896), the fixed obs
# tests and the plane-cached greedy; the ITER = 1 k_col2<16> exp build (soffset-0 stage stores)
# through the 256 tests + a mono timing A/B; then the rocprofv3 sets (trace + FETCH / WRITE / SQ /
# LDS passes) at N = 1024 and at the 896 crop, summarised on the box.
set -o pipefail
T=gpurun_out/r04b
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_obs.py tests/test_gpu_dbs_headline.py \
  -m gpu -v -k "896 or obs or graph or plane_cache or ratio05" --timeout 300 --timeout-method thread \
  > $T/gpu_tests_896.txt 2>&1
rc=$?
tail -3 $T/gpu_tests_896.txt
if [ $rc -gt 1 ]; then exit $rc; fi
HBX_LIB=$PWD/binary-hologram-reinforcement-learning_amd/hbx/libhbx_exp_COL2_ITER1.so timeout -k 10 300 \
  python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_planes.py -m gpu -v \
  -k "256 or mono or every_flip" --timeout 200 --timeout-method thread > $T/iter1_tests.txt 2>&1
irc=$?
tail -3 $T/iter1_tests.txt
if [ $irc -gt 1 ]; then exit $irc; fi
for lib in libhbx.so libhbx_exp_COL2_ITER1.so libhbx.so libhbx_exp_COL2_ITER1.so; do
  HBX_LIB=$PWD/binary-hologram-reinforcement-learning_amd/hbx/$lib timeout -k 10 200 python bench.py --steps 20 \
    --warmup 3 --cpu-sample 0 --dbs-flips 0 --no-probe --no-precision --no-obs --no-psf --no-planes \
    --no-psnr-check --no-scipy > $T/mono_$lib.json 2>> $T/mono.err || exit 20
  python3 -c "import json,sys; d=json.load(open('$T/mono_$lib.json')); m=d['ppo_mono_256']; c=d['crop_896']; print('$lib', d['value'], d['passes']['k_col']['avg_ms'], m['ms_per_step'], {k: v['avg_ms'] for k, v in m['passes'].items()}, 'crop', c['value'], {k: v['avg_ms'] for k, v in c['passes'].items()})" | tee -a $T/iter1_ab.txt
done
bash tools/profile.sh r04b > /dev/null || exit 10
python3 tools/pmc_summary.py gpurun_out/prof_r04b --jobs 128 --N 1024 --out gpurun_out/prof_r04b/pmc_summary.json \
  > gpurun_out/prof_r04b/pmc_summary.txt 2>&1 || exit 11
find gpurun_out/prof_r04b \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
bash tools/profile.sh r04b_896 --size 896 --no-ppo > /dev/null || exit 12
python3 tools/pmc_summary.py gpurun_out/prof_r04b_896 --jobs 128 --N 896 \
  --out gpurun_out/prof_r04b_896/pmc_summary.json > gpurun_out/prof_r04b_896/pmc_summary.txt 2>&1 || exit 13
find gpurun_out/prof_r04b_896 \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
python3 - <<'PY'
import json
for t in ("r04b", "r04b_896"):
    d = json.load(open(f"gpurun_out/prof_{t}/pmc_summary.json"))
    for k, v in d["kernels"].items():
        print(t, k, round(v["avg_ms"], 4), "alg", round(v["alg_GBs"] or 0), "hbm x",
              round((v["hbm_bytes_per_launch"] or 0) / (v["alg_bytes_per_launch"] or 1), 3),
              "bank", v.get("SQ_LDS_BANK_CONFLICT"), "vgpr", v.get("vgpr"))
PY
exit $rc

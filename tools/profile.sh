#!/bin/bash
# Kernel trace + PMC passes of a short bench run (run ON the GPU box, from the repo root).
# Usage: bash tools/profile.sh <tag> [bench args...]
# Each rocprofv3 pass is its own run (counters never combined with trace domains).
set -o pipefail
TAG=${1:-run}; shift
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="python3 bench.py --steps 6 --warmup 2 --psf-steps 20 --cpu-sample 0 --dbs-flips 0 --no-probe --no-psnr-check --no-precision --no-planes --no-crop --no-obs --no-dropin $*"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BENCH > $OUT/trace.log 2>&1 || exit 1
# headline-only trace: every FFT-mode pass launch is a 128-job step / reset chunk, so the
# --stats average of the dominant kernel is directly comparable with bench.py's roofline
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_headline -o run -- $BENCH --no-psf --no-ppo > $OUT/trace_headline.log 2>&1 || exit 6
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $BENCH > $OUT/fetch.log 2>&1 || exit 2
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $BENCH > $OUT/write.log 2>&1 || exit 3
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/sq -o run -- $BENCH > $OUT/sq.log 2>&1 || exit 4
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/lds -o run -- $BENCH > $OUT/lds.log 2>&1 || exit 5
python3 tools/pmc_summary.py $OUT --N ${PMC_N:-1024} --out $OUT/pmc_summary.json > /dev/null || exit 7
# the per-dispatch traces / counter rows are tens of MB: keep the summaries (the --stats csv
# and pmc_summary.json) so gpurun_out/ stays under the 64-MiB copy-back limit
find $OUT \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" -o -name "*agent_info.csv" \) -delete
find $OUT -name "*.csv" | head -40

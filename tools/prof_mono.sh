#!/bin/bash
# PMC passes of the 256x256x8 mono step (tools/pg_overhead.py, 4 x 20 steps); run ON the GPU box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof_mono_${1:-run}
mkdir -p $OUT
P="python3 tools/pg_overhead.py none 0 0 20"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $P > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $P > $OUT/fetch.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $P > $OUT/write.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/sq -o run -- $P > $OUT/sq.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/lds -o run -- $P > $OUT/lds.log 2>&1 || exit 5
python3 tools/pmc_summary.py $OUT --N 256 --out $OUT/pmc_summary.json > /dev/null || exit 7
# the per-dispatch traces / counter rows are tens of MB: keep the summaries (the --stats csv
# and pmc_summary.json) so gpurun_out/ stays under the 64-MiB copy-back limit
find $OUT \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" -o -name "*agent_info.csv" \) -delete
find $OUT -name "*.csv" | head -40

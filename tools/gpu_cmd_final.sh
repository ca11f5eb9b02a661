# Round-end evidence on one GPU: full -m gpu suite, default bench line, rocprofv3 trace + PMC passes.
set -o pipefail
T=${1:-r02_final2}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.txt 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err &&
bash tools/profile.sh $T
# summarise on the box and keep only the small files (the counter CSVs exceed gpurun's copy-back cap)
P=gpurun_out/prof_$T
python tools/pmc_summary.py $P --out gpurun_out/$T/pmc_summary.json > gpurun_out/$T/pmc_summary.txt 2>&1 &&
cp $P/trace/run_kernel_stats.csv gpurun_out/$T/kernel_stats.csv &&
cp $P/trace_headline/run_kernel_stats.csv gpurun_out/$T/kernel_stats_headline.csv &&
rm -rf $P

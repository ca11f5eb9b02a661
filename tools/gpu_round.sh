#!/bin/bash
# One GPU call: the -m gpu suite, then (unless it faulted / timed out) a short bench line.
#   bash tools/gpu_round.sh TAG [bench args...]
# Test failures (rc 1) still run the bench; any other non-zero status stops the call.
set -o pipefail
T=${1:-r03}
shift
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/$T/gpu_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/$T/gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
brc=$?
tail -c 3000 gpurun_out/$T/bench.json
exit $(( rc > brc ? rc : brc ))

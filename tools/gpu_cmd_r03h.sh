#!/bin/bash
# r03h: rocprofv3 kernel trace + PMC passes on HEAD (headline 1024x24 and 256x8 mono)
set -o pipefail
bash tools/profile.sh r03h || exit $?
bash tools/prof_mono.sh r03h || exit $?

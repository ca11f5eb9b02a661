#!/bin/bash
# r03i: iteration-count sweep with the non-temporal intermediate stores (k_col2 lines per lane
# group at N = 1024, k_rowfwd row blocks per workgroup at N = 1024 / 256)
set -o pipefail
bash tools/ab.sh r03i libhbx libhbx_exp_CIT32=2 libhbx_exp_CIT32=8 libhbx_exp_RIT32=2 libhbx_exp_RIT32=8 libhbx libhbx_exp_CIT32=8 libhbx_exp_RIT32=8 || exit 1
bash tools/ab_mono.sh libhbx libhbx_exp_RIT16=4 libhbx libhbx_exp_RIT16=4

#!/bin/bash
# r03n: s_setprio around k_col2's staged B stores (P2 / P3: priority 2 / 3) and, P2LD, also around
# its next-line A loads: headline timing A/B, builds alternated (r03n round 1 also measured
# SETPRIO_FWD around k_rowfwd32's A stores: no gain)
set -o pipefail
mkdir -p gpurun_out/r03n
bash tools/ab.sh r03n_ab2 libhbx libhbx_exp_P2 libhbx_exp_P3 libhbx_exp_P2LD \
  libhbx libhbx_exp_P2 libhbx_exp_P3 libhbx_exp_P2LD libhbx libhbx_exp_P2 libhbx_exp_P3 libhbx_exp_P2LD | tee gpurun_out/r03n/ab2.txt

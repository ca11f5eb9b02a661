#!/bin/bash
# r03o: the adopted setprio(2) k_col2 (libhbx) against the previous HEAD (OLD) at 1024x24 and 256x8,
# and setprio(2) around k_rowinv_d's plane loads (RINV_PRIO, on top of libhbx), builds alternated
set -o pipefail
mkdir -p gpurun_out/r03o
bash tools/ab.sh r03o_ab libhbx libhbx_exp_OLD libhbx_exp_RINV_PRIO libhbx libhbx_exp_OLD libhbx_exp_RINV_PRIO \
  libhbx libhbx_exp_OLD libhbx_exp_RINV_PRIO | tee gpurun_out/r03o/ab.txt || exit 1
bash tools/ab_mono.sh libhbx libhbx_exp_OLD libhbx_exp_RINV_PRIO libhbx libhbx_exp_OLD libhbx_exp_RINV_PRIO | tee gpurun_out/r03o/ab_mono.txt

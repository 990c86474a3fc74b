#!/bin/bash
# Binned-level split sweep (GPU): kbench of the scatter halves per MFNERF_BIN_LEVELS value.
set -o pipefail
mkdir -p gpurun_out
for k in ${LEVELS:-4 6 8 9}; do
  echo "== MFNERF_BIN_LEVELS=$k"
  MFNERF_BIN_LEVELS=$k timeout -k 10 180 python tools/kbench.py grid_bw grid_bw_coarse grid_bw_binned ${EXTRA} || exit 1
done

#!/bin/bash
# kbench of chosen stages per experiment build (GPU): VARIANTS="base c32" STAGES="grid_bw_coarse" ENVS="MFNERF_BIN_LEVELS=10"
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do for e in ${ENVS:-NONE=0}; do
  lib=mf-nerf_amd/libmfnerf_hip.so; [ "$v" = base ] || lib=mf-nerf_amd/csrc/var/libmfnerf_$v.so
  echo "== $v $e"
  env $e MFNERF_LIB=$lib timeout -k 10 180 python tools/kbench.py ${STAGES:-grid_bw} 2>&1 | grep -v amdgpu.ids || exit 1
done; done

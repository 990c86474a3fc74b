#!/bin/bash
# Scatter iteration (GPU): grid + engine tests, then kbench of the scatter stages and a short bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_field.py -k "grid_encode" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_grid.log 2>&1 || { tail -40 gpurun_out/t_grid.log; exit 1; }
tail -1 gpurun_out/t_grid.log
timeout -k 10 200 python tools/kbench.py grid_bw grid_bw_coarse grid_bw_binned adam_fixed 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu-baseline 2>/dev/null | cut -c1-200 || exit 1
[ -n "$VARIANTS" ] && { VARIANTS="$VARIANTS" STAGES="grid_bw grid_bw_binned" bash tools/sweep_variants.sh || exit 1; }
exit 0

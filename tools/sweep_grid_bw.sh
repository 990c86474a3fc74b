#!/bin/bash
# grid_bw launch-size x parts sweep of the bench (GPU).  Each run ~15 s.
set -o pipefail
mkdir -p gpurun_out
CFGS=${CFGS:-"1:4096 1:1024 1:512 2:4096 2:1024 2:512 2:256"}
for cfg in $CFGS; do
  cfg=${cfg/:/ }
  set -- $cfg
  MFNERF_GRID_BW_BLOCKS=$2 timeout -k 10 120 python bench.py --parts $1 --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/sw.json 2>/dev/null || exit 1
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/sw.json").read().strip().splitlines()[-1])
print(f"parts={sys.argv[1]} blocks={sys.argv[2]:>5}  ms/step {d['ms_per_step']:.4f}  grid_bw {d['grid_bw_ms']:.4f}  eager grid_bw {d['eager_stage_ms']['grid_bw']:.4f}", flush=True)
PY
done

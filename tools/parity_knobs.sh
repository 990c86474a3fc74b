#!/bin/bash
# training-parity test under scatter knob settings (GPU): prints the held-out PSNR line per setting
set -o pipefail
mkdir -p gpurun_out
for e in ${ENVS:-NONE=0}; do
  echo "== $e"
  env $e timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_train.py -x -q -s --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/pk.log 2>&1
  grep "held-out" gpurun_out/pk.log | cut -c1-200; tail -1 gpurun_out/pk.log
done

#!/bin/bash
# Benches of one build under several environment settings on one box (ENVS: space-separated
# NAME=VALUE words, "-" = none), twice each, after the GPU tests in $TESTS.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py} -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/abe_tests.log 2>&1 || { tail -30 gpurun_out/abe_tests.log; exit 1; }
tail -1 gpurun_out/abe_tests.log
for rep in 1 2; do
for E in $ENVS; do
  if [ "$E" = "-" ]; then ENV=""; else ENV="$E"; fi
  env $ENV timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup 30 --no-cpu-baseline > gpurun_out/abe.json 2> gpurun_out/abe.err || { tail -20 gpurun_out/abe.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abe.json'));print('$E',d['ms_per_step'],d['grid_bw_ms'])"
done
done

#!/bin/bash
# Benches of several library builds on one box (LIBS: space-separated paths, "-" = the default build), twice each.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py} -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/abl_tests.log 2>&1 || { tail -30 gpurun_out/abl_tests.log; exit 1; }
tail -1 gpurun_out/abl_tests.log
for rep in 1 2; do
for L in $LIBS; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/$L; fi
  timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup 30 --no-cpu-baseline > gpurun_out/abl.json 2> gpurun_out/abl.err || { tail -20 gpurun_out/abl.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abl.json'));print('$L',d['ms_per_step'],d['grid_bw_ms'])"
done
done

#!/bin/bash
# A/B of two library builds: engine GPU tests on B, then alternating benches of A (default) and B.
set -o pipefail
mkdir -p gpurun_out
B=${B:-mf-nerf_amd/csrc/var/libmfnerf_pair.so}
MFNERF_LIB=$PWD/$B timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_field.py tests/test_gpu_engine.py} -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for v in A B A B; do
  if [ $v = B ]; then export MFNERF_LIB=$PWD/$B; else unset MFNERF_LIB; fi
  timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup 30 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -20 gpurun_out/ab_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v',d['ms_per_step'],d['grid_bw_ms'],d['eager_stage_ms']['field_bw'])"
done

#!/bin/bash
# Planar encode with both levels' gathers in flight: parity + timings + bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_golden.py tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s15_tests.log 2>&1 && \
timeout -k 10 120 python tools/kbench.py grid_fw_planar > gpurun_out/s15_kb0.log 2>&1 && \
MFNERF_KBENCH_PRESET=mf128 timeout -k 10 120 python tools/kbench.py grid_fw_planar > gpurun_out/s15_kb2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/s15_bench.json 2> gpurun_out/s15_bench.err
rc=$?
echo "EXIT $rc"; tail -n 3 gpurun_out/s15_tests.log; grep grid_fw gpurun_out/s15_kb0.log gpurun_out/s15_kb2.log; cut -c1-300 gpurun_out/s15_bench.json
exit $rc

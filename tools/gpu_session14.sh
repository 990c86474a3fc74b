#!/bin/bash
# level_l1 zeroed by the Adam bump kernel; phased planar encode A/B; parity + bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_field.py tests/test_gpu_train.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s14_tests.log 2>&1 && \
timeout -k 10 120 python tools/kbench.py grid_fw_planar > gpurun_out/s14_kb0.log 2>&1 && \
MFNERF_GRID_FW_PHASED=1 timeout -k 10 120 python tools/kbench.py grid_fw_planar > gpurun_out/s14_kb1.log 2>&1 && \
MFNERF_KBENCH_PRESET=mf128 timeout -k 10 120 python tools/kbench.py grid_fw_planar > gpurun_out/s14_kb2.log 2>&1 && \
MFNERF_KBENCH_PRESET=mf128 MFNERF_GRID_FW_PHASED=1 timeout -k 10 120 python tools/kbench.py grid_fw_planar > gpurun_out/s14_kb3.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/s14_bench.json 2> gpurun_out/s14_bench.err
rc=$?
echo "EXIT $rc"; tail -3 gpurun_out/s14_tests.log; tail -1 gpurun_out/s14_kb0.log gpurun_out/s14_kb1.log gpurun_out/s14_kb2.log gpurun_out/s14_kb3.log; cut -c1-300 gpurun_out/s14_bench.json
exit $rc

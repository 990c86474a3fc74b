#!/bin/bash
# AGPR-pinned weight-gradient accumulators: field parity + per-kernel timing of field_bw (both presets).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/s7_tests.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py field_bw field_fw > gpurun_out/s7_kb64.log 2>&1 && \
MFNERF_KBENCH_PRESET=mf128 timeout -k 10 300 python tools/kbench.py field_bw field_fw > gpurun_out/s7_kb128.log 2>&1
rc=$?
echo "EXIT $rc"; tail -3 gpurun_out/s7_tests.log; cat gpurun_out/s7_kb64.log gpurun_out/s7_kb128.log 2>/dev/null | tail -12
exit $rc

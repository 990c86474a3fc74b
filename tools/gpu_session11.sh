#!/bin/bash
# MLP weight-gradient fold on a second stream beside grid_bw: engine/train/dp parity, bench both presets.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/diag_replay.py > gpurun_out/s11_diag.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_train.py tests/test_gpu_field.py tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s11_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/s11_bench.json 2> gpurun_out/s11_bench.err && \
timeout -k 10 300 python bench.py --preset mf128 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/s11_bench128.json 2> gpurun_out/s11_bench128.err
rc=$?
echo "EXIT $rc"; grep -v amdgpu.ids gpurun_out/s11_diag.log; tail -15 gpurun_out/s11_tests.log; cat gpurun_out/s11_bench.json gpurun_out/s11_bench128.json 2>/dev/null | cut -c1-400
exit $rc

#!/bin/bash
# Fused fixed-point convert + Adam: engine/train parity, then the bench (lego, mf128).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s8_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/s8_bench.json 2> gpurun_out/s8_bench.err && \
timeout -k 10 300 python bench.py --preset mf128 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/s8_bench128.json 2> gpurun_out/s8_bench128.err
rc=$?
echo "EXIT $rc"; tail -3 gpurun_out/s8_tests.log; cat gpurun_out/s8_bench.json gpurun_out/s8_bench128.json 2>/dev/null; tail -3 gpurun_out/s8_bench.err
exit $rc

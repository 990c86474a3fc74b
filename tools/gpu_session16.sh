#!/bin/bash
# Optimizer tail deferred into the next chain graph: all GPU tests, bench both presets, timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/s16_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/s16_bench.json 2> gpurun_out/s16_bench.err && \
timeout -k 10 300 python bench.py --preset mf128 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/s16_bench128.json 2> gpurun_out/s16_bench128.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof16 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/prof16.log 2>&1
rc=$?
echo "EXIT $rc"; tail -n 3 gpurun_out/s16_tests.log; cut -c1-300 gpurun_out/s16_bench.json gpurun_out/s16_bench128.json
python3 tools/step_timeline.py gpurun_out/prof16/run_kernel_trace.csv
exit $rc

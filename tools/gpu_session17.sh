#!/bin/bash
# Round-1 final state: all GPU tests, the default bench line (with the CPU baseline), mf128, kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/s17_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/s17_bench.json 2> gpurun_out/s17_bench.err && \
timeout -k 10 300 python bench.py --preset mf128 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/s17_bench128.json 2> gpurun_out/s17_bench128.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof17 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/prof17.log 2>&1
rc=$?
echo "EXIT $rc"; tail -n 3 gpurun_out/s17_tests.log; cut -c1-300 gpurun_out/s17_bench.json gpurun_out/s17_bench128.json
python3 tools/step_timeline.py gpurun_out/prof17/run_kernel_trace.csv > gpurun_out/s17_timeline.txt
exit $rc

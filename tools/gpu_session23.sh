#!/bin/bash
# Marched-sample count accumulated in one op on the side chain: engine tests, bench, timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s23_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s23_bench.json 2> gpurun_out/s23_b.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s23_bench_b.json 2> gpurun_out/s23_bb.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof23 -o run --output-format csv -- python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/prof23.log 2>&1
rc=$?
echo "EXIT $rc"; tail -n 2 gpurun_out/s23_tests.log; cut -c1-200 gpurun_out/s23_bench.json gpurun_out/s23_bench_b.json
python3 tools/step_timeline.py gpurun_out/prof23/run_kernel_trace.csv > gpurun_out/s23_timeline.txt
exit $rc

#!/bin/bash
# Scatter + Adam tail replayed as one graph: engine/train tests, bench with the scatter timed on every
# step (old layout) vs every 8th, mf128, kernel trace timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s20_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --roofline-every 1 > gpurun_out/s20_bench_every1.json 2> gpurun_out/s20_b1.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s20_bench.json 2> gpurun_out/s20_b.err && \
timeout -k 10 300 python bench.py --preset mf128 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/s20_bench128.json 2> gpurun_out/s20_b128.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof20 -o run --output-format csv -- python3 bench.py --steps 32 --warmup 10 --no-cpu-baseline > gpurun_out/prof20.log 2>&1
rc=$?
echo "EXIT $rc"; tail -n 3 gpurun_out/s20_tests.log; cut -c1-260 gpurun_out/s20_bench_every1.json gpurun_out/s20_bench.json gpurun_out/s20_bench128.json
python3 tools/step_timeline.py gpurun_out/prof20/run_kernel_trace.csv > gpurun_out/s20_timeline.txt
exit $rc

#!/bin/bash
# Next step's march issued at the step's start (beside the chain) vs under grid_bw.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MFNERF_MARCH_EARLY=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s21_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s21_bench0.json 2> gpurun_out/s21_b0.err && \
MFNERF_MARCH_EARLY=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s21_bench1.json 2> gpurun_out/s21_b1.err && \
MFNERF_MARCH_EARLY=1 timeout -k 10 300 python bench.py --preset mf128 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/s21_bench128.json 2> gpurun_out/s21_b128.err && \
MFNERF_MARCH_EARLY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof21 -o run --output-format csv -- python3 bench.py --steps 32 --warmup 10 --no-cpu-baseline > gpurun_out/prof21.log 2>&1
rc=$?
echo "EXIT $rc"; tail -n 3 gpurun_out/s21_tests.log; cut -c1-200 gpurun_out/s21_bench0.json gpurun_out/s21_bench1.json gpurun_out/s21_bench128.json
python3 tools/step_timeline.py gpurun_out/prof21/run_kernel_trace.csv > gpurun_out/s21_timeline.txt
exit $rc

#!/bin/bash
# Deterministic field_bw epilogue + float4 slab reduce: parity, determinism, timings, bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_field.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s13_tests.log 2>&1 && \
timeout -k 10 120 python tools/kbench.py field_bw adam adam_fixed > gpurun_out/s13_kb.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/s13_bench.json 2> gpurun_out/s13_bench.err && \
timeout -k 10 300 python bench.py --preset mf128 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/s13_bench128.json 2> gpurun_out/s13_bench128.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof14 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/prof14.log 2>&1
rc=$?
echo "EXIT $rc"; tail -3 gpurun_out/s13_tests.log; tail -4 gpurun_out/s13_kb.log; cat gpurun_out/s13_bench.json gpurun_out/s13_bench128.json 2>/dev/null | cut -c1-300
python3 tools/step_timeline.py gpurun_out/prof14/run_kernel_trace.csv
exit $rc

#!/bin/bash
# DPP wave-shift transmittance chain: compositing parity (bit-exact vs oracle), golden, engine; timings.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_vren.py tests/test_gpu_golden.py tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s10_tests.log 2>&1 && \
timeout -k 10 120 python tools/kbench.py composite composite_fw composite_bw > gpurun_out/s10_kb.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/s10_bench.json 2> gpurun_out/s10_bench.err
rc=$?
echo "EXIT $rc"; tail -3 gpurun_out/s10_tests.log; tail -4 gpurun_out/s10_kb.log; cat gpurun_out/s10_bench.json
exit $rc

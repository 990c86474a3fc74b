#!/bin/bash
# Targeted GPU tests (TESTS) then a bench (STEPS), each under its own time limit, chained with &&.
set -o pipefail
mkdir -p gpurun_out
TESTS=${TESTS:-tests/test_gpu_field.py}
timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/quick_tests.log 2>&1 || { tail -40 gpurun_out/quick_tests.log; exit 1; }
tail -2 gpurun_out/quick_tests.log
timeout -k 10 400 python bench.py --steps ${STEPS:-300} --warmup 30 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err || { tail -20 gpurun_out/quick_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/quick_bench.json'));print(d['ms_per_step'],d['value'],d['grid_bw_ms'],d['eager_stage_ms'])"

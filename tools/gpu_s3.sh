#!/bin/bash
# Targeted tests, a bench, and one profiled bench's step timeline (the fused one-graph steps).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_vren.py tests/test_gpu_engine.py} -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s3_tests.log 2>&1 || { tail -40 gpurun_out/s3_tests.log; exit 1; }
tail -1 gpurun_out/s3_tests.log
timeout -k 10 400 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/s3_bench.json 2> gpurun_out/s3_bench.err || { tail -20 gpurun_out/s3_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/s3_bench.json'));print(d['ms_per_step'],d['value'],d['grid_bw_ms'],d['eager_stage_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/prof3.log 2>&1 || { tail -20 gpurun_out/prof3.log; exit 1; }
python tools/step_timeline.py gpurun_out/prof3 --last 1 | head -20

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vren.py tests/test_gpu_engine.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s2_tests.log 2>&1 || { tail -40 gpurun_out/s2_tests.log; exit 1; }
tail -1 gpurun_out/s2_tests.log
timeout -k 10 400 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/s2_bench.json 2> gpurun_out/s2_bench.err || { tail -20 gpurun_out/s2_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/s2_bench.json'));print(d['ms_per_step'],d['value'],d['grid_bw_ms'],d['eager_stage_ms'])"
bash tools/gpu_pmc.sh > gpurun_out/pmc.out 2>&1 || { tail -20 gpurun_out/pmc.out; exit 1; }
python tools/step_timeline.py gpurun_out/prof --last 1 | head -20

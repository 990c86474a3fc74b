#!/bin/bash
# One GPU session: parity tests, smoke, bench (both presets), render FPS, rocprof kernel stats.
# Every GPU step has its own time limit and the steps are chained with && (a failure ends it).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-100}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps $STEPS --warmup 20 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 600 python bench.py --preset mf128 --steps 50 --warmup 10 > gpurun_out/bench_mf128.json 2> gpurun_out/bench_mf128.err && \
timeout -k 10 600 python tools/render_fps.py > gpurun_out/render_fps.json 2> gpurun_out/render_fps.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?
echo "EXIT $rc"
tail -5 gpurun_out/gpu_tests.log; cat gpurun_out/smoke.log 2>/dev/null | tail -3; cat gpurun_out/bench.json gpurun_out/bench_mf128.json gpurun_out/render_fps.json 2>/dev/null; tail -3 gpurun_out/bench.err gpurun_out/render_fps.err 2>/dev/null
exit $rc

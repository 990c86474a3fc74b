#!/bin/bash
# Round-end state: all GPU tests, smoke(), the default bench line (CPU baseline included), kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/s22_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/s22_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/s22_bench.json 2> gpurun_out/s22_bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof22 -o run --output-format csv -- python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/prof22.log 2>&1
rc=$?
echo "EXIT $rc"; tail -n 2 gpurun_out/s22_tests.log; tail -n 1 gpurun_out/s22_smoke.log; cut -c1-300 gpurun_out/s22_bench.json
python3 tools/step_timeline.py gpurun_out/prof22/run_kernel_trace.csv > gpurun_out/s22_timeline.txt
exit $rc

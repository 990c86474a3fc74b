set -o pipefail
mkdir -p gpurun_out/r4a
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.err && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_dp_replay.py "tests/test_gpu_tcnn.py::test_sh4_fw_kernel_matches_the_oracle" > gpurun_out/r4a/tests.log 2>&1 && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4a/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --roofline-every 1 > $GRAFT_REPO_ROOT/gpurun_out/r4a/prof.log 2>&1 && cd $GRAFT_REPO_ROOT && \
python tools/step_timeline.py gpurun_out/r4a/prof > gpurun_out/r4a/timeline.txt && \
STAGE=grid_bw timeout -k 10 400 bash tools/pmc_sq.sh

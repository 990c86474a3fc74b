set -o pipefail
mkdir -p gpurun_out/r4a
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_field.py::test_staged_accumulate_matches_per_slot_form "tests/test_gpu_field.py::test_grid_encode_fw_bw" tests/test_gpu_engine.py::test_large_tables_train_with_or_without_partitions tests/test_gpu_engine.py::test_timed_and_fused_tail_replays_match_eager tests/test_gpu_occupancy.py tests/test_gpu_dp_replay.py "tests/test_gpu_tcnn.py::test_sh4_fw_kernel_matches_the_oracle" > gpurun_out/r4a/tests.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.err && \
MFNERF_ACCUM=0 timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/r4a/bench_acc0.json 2> gpurun_out/r4a/bench_acc0.err && \
timeout -k 10 200 python tools/kbench.py grid_bw grid_bw_fused occupancy grid_fw_planar field_bw > gpurun_out/r4a/kbench.txt 2>&1 && \
MFNERF_ACCUM=0 timeout -k 10 200 python tools/kbench.py grid_bw grid_bw_fused > gpurun_out/r4a/kbench_acc0.txt 2>&1 && \
MFNERF_SCATTER_HALVES=2 timeout -k 10 200 python tools/kbench.py grid_bw grid_bw_fused > gpurun_out/r4a/kbench_h2.txt 2>&1 && \
MFNERF_SCATTER_HALVES=2 timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/r4a/bench_h2.json 2> gpurun_out/r4a/bench_h2.err && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4a/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --roofline-every 1 > $GRAFT_REPO_ROOT/gpurun_out/r4a/prof.log 2>&1 && cd $GRAFT_REPO_ROOT && \
python tools/step_timeline.py gpurun_out/r4a/prof > gpurun_out/r4a/timeline.txt && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4a/prof_occ -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kbench.py occupancy > $GRAFT_REPO_ROOT/gpurun_out/r4a/prof_occ.log 2>&1 && cd $GRAFT_REPO_ROOT && \
STAGE=grid_bw timeout -k 10 400 bash tools/pmc_sq.sh

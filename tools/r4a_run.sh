set -o pipefail
mkdir -p gpurun_out/r4a
export TMPDIR=/tmp
export MFNERF_PARITY_OUT=$GRAFT_REPO_ROOT/gpurun_out/r4a/parity_train.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4a/tests.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.err && \
MFNERF_ACCUM=0 timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/r4a/bench_acc0.json 2> gpurun_out/r4a/bench_acc0.err && \
MFNERF_SCATTER_HALVES=2 timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/r4a/bench_h2.json 2> gpurun_out/r4a/bench_h2.err && \
timeout -k 10 200 python tools/kbench.py grid_bw grid_bw_fused occupancy grid_fw_planar field_bw > gpurun_out/r4a/kbench.txt 2>&1 && \
MFNERF_ACCUM=0 timeout -k 10 200 python tools/kbench.py grid_bw grid_bw_fused > gpurun_out/r4a/kbench_acc0.txt 2>&1 && \
MFNERF_SCATTER_HALVES=2 timeout -k 10 200 python tools/kbench.py grid_bw grid_bw_fused > gpurun_out/r4a/kbench_h2.txt 2>&1 && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4a/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --roofline-every 1 > $GRAFT_REPO_ROOT/gpurun_out/r4a/prof.log 2>&1 && cd $GRAFT_REPO_ROOT && \
python tools/step_timeline.py gpurun_out/r4a/prof > gpurun_out/r4a/timeline.txt && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4a/prof_occ -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kbench.py occupancy > $GRAFT_REPO_ROOT/gpurun_out/r4a/prof_occ.log 2>&1 && cd $GRAFT_REPO_ROOT && \
timeout -k 10 200 python bench.py --steps 100 --warmup 20 --dp-rehearse --no-cpu-baseline > gpurun_out/r4a/bench_dp.json 2> gpurun_out/r4a/bench_dp.err && \
MFNERF_DIRECT_RCCL=0 timeout -k 10 200 python bench.py --steps 100 --warmup 20 --dp-rehearse --no-cpu-baseline > gpurun_out/r4a/bench_dp_torch.json 2> gpurun_out/r4a/bench_dp_torch.err && \
STAGE=grid_bw timeout -k 10 400 bash tools/pmc_sq.sh

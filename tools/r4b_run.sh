set -o pipefail
mkdir -p gpurun_out/r4b
export TMPDIR=/tmp
export MFNERF_PARITY_OUT=$GRAFT_REPO_ROOT/gpurun_out/r4b/parity_train.json
# a step may fail (exit 1: a test or an assertion) and the next still run; anything else (abort,
# fault, time limit) ends the script
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 200 python tools/diag_occ.py > gpurun_out/r4b/diag_occ.log 2>&1; ok
MFNERF_OCC_GRAPH=0 timeout -k 10 200 python tools/diag_occ.py > gpurun_out/r4b/diag_occ_eager.log 2>&1; ok
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_occupancy.py::test_engine_refresh_end_to_end > gpurun_out/r4b/tests.log 2>&1; ok
timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/r4b/bench.json 2> gpurun_out/r4b/bench.err && \
MFNERF_FIELD_BW_COOP=0 timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/r4b/bench_nocoop.json 2> gpurun_out/r4b/bench_nocoop.err && \
MFNERF_ACCUM=0 MFNERF_FIELD_BW_COOP=0 timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/r4b/bench_acc0.json 2> gpurun_out/r4b/bench_acc0.err && \
MFNERF_SCATTER_HALVES=2 timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/r4b/bench_h2.json 2> gpurun_out/r4b/bench_h2.err && \
timeout -k 10 200 python tools/kbench.py grid_bw grid_bw_fused occupancy grid_fw_planar field_bw > gpurun_out/r4b/kbench.txt 2>&1 && \
MFNERF_FIELD_BW_COOP=0 MFNERF_ACCUM=0 timeout -k 10 200 python tools/kbench.py grid_bw grid_bw_fused field_bw > gpurun_out/r4b/kbench_old.txt 2>&1 && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4b/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --roofline-every 1 > $GRAFT_REPO_ROOT/gpurun_out/r4b/prof.log 2>&1 && cd $GRAFT_REPO_ROOT && \
python tools/step_timeline.py gpurun_out/r4b/prof > gpurun_out/r4b/timeline.txt

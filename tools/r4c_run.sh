set -o pipefail
mkdir -p gpurun_out/r4c
export TMPDIR=/tmp
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 200 python tools/diag_occ.py --poison > gpurun_out/r4c/diag_occ_poison.log 2>&1; ok
MFNERF_OCC_GRAPH=0 timeout -k 10 200 python tools/diag_occ.py --poison > gpurun_out/r4c/diag_occ_poison_eager.log 2>&1; ok
timeout -k 10 600 python -u -m pytest tests/test_gpu_occupancy.py tests/test_gpu_field.py tests/test_gpu_engine.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4c/tests.log 2>&1; ok
for G in composite field_fw grid_fw field_bw; do
  MFNERF_GATE_AT=$G timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/r4c/bench_gate_$G.json 2> gpurun_out/r4c/bench_gate_$G.err || exit $?
done
MFNERF_SCAN_WAVES=1 timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/r4c/bench_scan1.json 2> gpurun_out/r4c/bench_scan1.err && \
MFNERF_FIELD_BW_COOP=0 timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/r4c/bench_nocoop.json 2> gpurun_out/r4c/bench_nocoop.err && \
timeout -k 10 200 python tools/kbench.py grid_bw grid_fw_planar occupancy field_bw > gpurun_out/r4c/kbench.txt 2>&1 && \
MFNERF_SCAN_WAVES=1 timeout -k 10 200 python tools/kbench.py grid_bw > gpurun_out/r4c/kbench_scan1.txt 2>&1

set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_vren.py tests/test_gpu_golden.py tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t1.log 2>&1 && \
MFNERF_FIELD_BW_WAVES=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_field.py -k "field_bw or planar" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t8.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py > gpurun_out/kb4.log 2>&1 && \
MFNERF_FIELD_BW_WAVES=8 timeout -k 10 300 python tools/kbench.py field_bw > gpurun_out/kb8.log 2>&1 && \
MFNERF_KBENCH_PRESET=mf128 timeout -k 10 300 python tools/kbench.py > gpurun_out/kbmf.log 2>&1
rc=$?
echo "EXIT $rc"; tail -3 gpurun_out/t1.log; tail -3 gpurun_out/t8.log 2>/dev/null; cat gpurun_out/kb4.log gpurun_out/kb8.log gpurun_out/kbmf.log 2>/dev/null | grep -v "^$" | tail -60
exit $rc

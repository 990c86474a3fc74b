set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t3.log 2>&1 && \
MFNERF_KBENCH_PRESET=mf128 timeout -k 10 300 python tools/kbench.py field_fw field_bw grid_fw_planar grid_bw composite adam > gpurun_out/kbmf.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py field_bw > gpurun_out/kb4.log 2>&1
rc=$?
echo "EXIT $rc"; tail -3 gpurun_out/t3.log; cat gpurun_out/kbmf.log gpurun_out/kb4.log 2>/dev/null | grep -v "amdgpu.ids" | tail -30
exit $rc

set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MFNERF_FIELD_BW_WAVES=8 timeout -k 10 300 python tools/kbench.py field_bw composite > gpurun_out/kb8.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py field_bw adam pack march > gpurun_out/kb4b.log 2>&1 && \
MFNERF_KBENCH_PRESET=mf128 timeout -k 10 300 python tools/kbench.py > gpurun_out/kbmf.log 2>&1
rc=$?
echo "EXIT $rc"; cat gpurun_out/kb8.log gpurun_out/kb4b.log gpurun_out/kbmf.log 2>/dev/null | grep -v "amdgpu.ids" | tail -60
exit $rc

set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_field.py tests/test_gpu_train.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/t6.log 2>&1 && \
timeout -k 10 600 python tools/render_fps.py > gpurun_out/render_fps6.json 2> gpurun_out/render_fps6.err
rc=$?
echo "EXIT $rc"; tail -3 gpurun_out/t6.log; cat gpurun_out/render_fps6.json; tail -3 gpurun_out/render_fps6.err
exit $rc

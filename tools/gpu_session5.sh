set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_engine.py tests/test_gpu_dp.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/t5.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/bench5.json 2> gpurun_out/bench5.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/prof5.log 2>&1
rc=$?
echo "EXIT $rc"; tail -3 gpurun_out/t5.log; cat gpurun_out/bench5.json; tail -3 gpurun_out/bench5.err
exit $rc

set -o pipefail
D=gpurun_out/r4d
mkdir -p $D
export TMPDIR=/tmp
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1; ok
timeout -k 10 200 python tools/kbench.py grid_bw > $D/kbench_direct.txt 2>&1 || exit $?
MFNERF_SCATTER_NT=1 timeout -k 10 200 python tools/kbench.py grid_bw > $D/kbench_direct_nt.txt 2>&1 || exit $?
MFNERF_SCATTER_DIRECT=0 timeout -k 10 200 python tools/kbench.py grid_bw > $D/kbench_sorted.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > $D/bench_direct.json 2> $D/bench_direct.err || exit $?
MFNERF_SCATTER_NT=1 timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > $D/bench_direct_nt.json 2> $D/bench_direct_nt.err || exit $?
MFNERF_SCATTER_DIRECT=0 timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > $D/bench_sorted.json 2> $D/bench_sorted.err || exit $?
MFNERF_GATE_AT=field_bw timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > $D/bench_direct_gfb.json 2> $D/bench_direct_gfb.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python tools/kbench.py grid_bw > $D/prof.log 2>&1 || exit $?

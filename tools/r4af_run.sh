# DP step trimming: sharded Adam reads the exchanged flag and zeroes level_l1 itself.
set -o pipefail
D=gpurun_out/r4af
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_dp_replay.py tests/test_gpu_train.py tests/test_gpu_optim.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $D/bench.json 2> $D/bench.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --dp-rehearse > $D/bench_dp.json 2> $D/bench_dp.err || exit $?
MFNERF_DP_SHARD_ADAM=0 timeout -k 10 300 python bench.py --no-cpu-baseline --dp-rehearse > $D/bench_dp_unfused.json 2> $D/bench_dp_unfused.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_dp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --dp-rehearse > $GRAFT_REPO_ROOT/$D/prof_dp.log 2>&1 && cd $GRAFT_REPO_ROOT || exit $?
python tools/step_timeline.py $D/prof_dp > $D/timeline_dp.txt

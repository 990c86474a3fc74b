# Round-4 closing evidence of the committed tree: full GPU suite, smoke, bench lines (lego, mf128,
# T20, DP rehearsal), kernel stats + step timelines (N=1 and DP), 30k-step protocol.
set -o pipefail
D=gpurun_out/r4fin2
mkdir -p $D
export TMPDIR=/tmp
export MFNERF_PARITY_OUT=$GRAFT_REPO_ROOT/$D/parity_train.json
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1; ok
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $D/bench.json 2> $D/bench.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --preset mf128 > $D/bench_mf128.json 2> $D/bench_mf128.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --log2-T 20 > $D/bench_T20.json 2> $D/bench_T20.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --dp-rehearse > $D/bench_dp_rehearse.json 2> $D/bench_dp_rehearse.err || exit $?
timeout -k 10 400 python tools/train_30k.py > $D/train30k.json 2> $D/train30k.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 && cd $GRAFT_REPO_ROOT || exit $?
python tools/step_timeline.py $D/prof > $D/timeline.txt; ok
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_dp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --dp-rehearse > $GRAFT_REPO_ROOT/$D/prof_dp.log 2>&1 && cd $GRAFT_REPO_ROOT || exit $?
python tools/step_timeline.py $D/prof_dp > $D/timeline_dp.txt; ok

# Round-4 validation of the committed tree: full GPU suite, smoke, bench lines, kernel stats.
set -o pipefail
D=gpurun_out/r4y
mkdir -p $D
export TMPDIR=/tmp
export MFNERF_PARITY_OUT=$GRAFT_REPO_ROOT/$D/parity_train.json
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1; ok
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $D/bench.json 2> $D/bench.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --dp-rehearse > $D/bench_dp_rehearse.json 2> $D/bench_dp_rehearse.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 && cd $GRAFT_REPO_ROOT || exit $?
python tools/step_timeline.py $D/prof > $D/timeline.txt

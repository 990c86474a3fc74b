# DP step without the gradient-prefix fill (store-mode weight-gradient fold): tests + A/B.
set -o pipefail
D=gpurun_out/r4ai
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_dp.py tests/test_gpu_dp_replay.py tests/test_gpu_engine.py tests/test_gpu_optim.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $D/bench.json 2> $D/bench.err || exit $?
for k in 1 0 1 0; do
  MFNERF_DP_STORE_FOLD=$k timeout -k 10 300 python bench.py --no-cpu-baseline --dp-rehearse > $D/bench_dp_$k.json 2> $D/bench_dp_$k.err || exit $?
  python -c "import json; d=json.loads(open('$D/bench_dp_$k.json').read().strip().splitlines()[-1]); print('store_fold=$k', d['ms_per_step'])" | tee -a $D/summary.txt
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_dp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --dp-rehearse > $GRAFT_REPO_ROOT/$D/prof_dp.log 2>&1 && cd $GRAFT_REPO_ROOT || exit $?
python tools/step_timeline.py $D/prof_dp > $D/timeline_dp.txt

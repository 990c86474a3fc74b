# DP step with the shard flag folded into the float finish: tests + A/B.
set -o pipefail
D=gpurun_out/r4ak
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_dp.py tests/test_gpu_dp_replay.py tests/test_gpu_engine.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $D/bench.json 2> $D/bench.err || exit $?
for k in 1 0 1 0; do
  MFNERF_DP_FLAG_FOLD=$k timeout -k 10 300 python bench.py --no-cpu-baseline --dp-rehearse > $D/bench_dp_$k.json 2> $D/bench_dp_$k.err || exit $?
  python -c "import json; d=json.loads(open('$D/bench_dp_$k.json').read().strip().splitlines()[-1]); print('flag_fold=$k', d['ms_per_step'])" | tee -a $D/summary.txt
done
python -c "import json; d=json.loads(open('$D/bench.json').read().strip().splitlines()[-1]); print('N1', d['ms_per_step'])" | tee -a $D/summary.txt

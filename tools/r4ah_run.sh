# A/B: the step's stream at high queue priority vs the default stream (march on a normal side stream).
set -o pipefail
D=gpurun_out/r4ah
mkdir -p $D
export TMPDIR=/tmp
for k in 0 1 0 1 0 1; do
  MFNERF_MAIN_HIGH_PRIORITY=$k timeout -k 10 200 python bench.py --no-cpu-baseline > $D/bench_$k.json 2> $D/bench_$k.err || exit $?
  python -c "import json; d=json.loads(open('$D/bench_$k.json').read().strip().splitlines()[-1]); print('$k', d['ms_per_step'], d['grid_bw_ms'])" | tee -a $D/summary.txt
done

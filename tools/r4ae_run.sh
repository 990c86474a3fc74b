# A/B: planar encode workgroups per level group (refresh encode of ~628k points vs the step's ~490k).
set -o pipefail
D=gpurun_out/r4ae
mkdir -p $D
export TMPDIR=/tmp
for c in 2048 4096 8192 2048 4096 8192; do
  MFNERF_ENC_GROUP_CAP=$c timeout -k 10 200 python bench.py --no-cpu-baseline > $D/bench_$c.json 2> $D/bench_$c.err || exit $?
  python -c "import json,sys; d=json.loads(open('$D/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['ms_per_step'], d['density_update_ms'], d['eager_stage_ms']['grid_fw'])" | tee -a $D/summary.txt
done

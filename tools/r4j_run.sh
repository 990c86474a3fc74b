set -o pipefail
D=gpurun_out/r4j
mkdir -p $D
export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --roofline-every 1000"
for rep in 1 2; do
for V in "composite 1" "grid_fw 2" "grid_fw 3" "field_fw 2" "grid_fw 1"; do
  set -- $V
  MFNERF_GATE_AT=$1 MFNERF_MARCH_RPW=$2 $B > $D/ab.json 2> $D/ab.err || exit $?
  python -c "import json;d=json.load(open('$D/ab.json'));print('gate=$1 rpw=$2',d['ms_per_step'],d['grid_bw_ms'])" >> $D/ab.txt
done
done
cd /tmp && MFNERF_GATE_AT=grid_fw MFNERF_MARCH_RPW=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --roofline-every 1000 > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 && cd $GRAFT_REPO_ROOT && \
python tools/step_timeline.py $D/prof > $D/timeline.txt

# r5o (v2: F=2 a 40 MB copy forked beside the step, F=3 the same copy serial): cost of a forked stream inside the captured data-parallel graph (MFNERF_FORK_TEST=1: an
# in-place one-rank reduce-scatter of the first 983040 values on a second stream, joined before the
# exchange) -- the dp-rehearse bench with and without it, twice; a profiled timeline of the forked form.
set -o pipefail
D=gpurun_out/r5o
mkdir -p $D
export TMPDIR=/tmp
for rep in 1 2; do
for F in 0 2 3; do
  MFNERF_FORK_TEST=$F timeout -k 10 200 python bench.py --dp-rehearse --steps 300 --warmup 30 --no-cpu-baseline > $D/b_$F.json 2> $D/b_$F.err || { tail -20 $D/b_$F.err; exit 1; }
  python -c "import json;d=json.load(open('$D/b_$F.json'));print('fork=$F',d['ms_per_step'],d['config'].get('exchange'))"
done
done
cd /tmp && MFNERF_FORK_TEST=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --dp-rehearse --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1; cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $D/prof > $D/timeline.txt && cat $D/timeline.txt

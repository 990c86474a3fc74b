# r5y: round-5 closing evidence, part 2 (GPU box): the bench's kernel stats + step timeline (default and
# the data-parallel rehearsal), PMC traffic / MFMA busy of the mf128 preset, SQ issue profiles of
# grid_bw and field_bw (tools/pmc_sq.sh).
set -o pipefail
D=gpurun_out/r5y
mkdir -p $D
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 && cd $GRAFT_REPO_ROOT || exit $?
python3 tools/step_timeline.py $D/prof > $D/timeline.txt && cat $D/timeline.txt | head -3
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_dp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --dp-rehearse > $GRAFT_REPO_ROOT/$D/prof_dp.log 2>&1 && cd $GRAFT_REPO_ROOT || exit $?
python3 tools/step_timeline.py $D/prof_dp > $D/timeline_dp.txt && head -1 $D/timeline_dp.txt
PRESET=mf128 timeout -k 10 500 bash tools/gpu_pmc.sh > $D/pmc_mf128.log 2>&1 || { tail -20 $D/pmc_mf128.log; exit 1; }
STAGE=grid_bw timeout -k 10 400 bash tools/pmc_sq.sh > $D/sq_grid_bw.log 2>&1 || { tail -20 $D/sq_grid_bw.log; exit 1; }
STAGE=field_bw timeout -k 10 400 bash tools/pmc_sq.sh > $D/sq_field_bw.log 2>&1 || { tail -20 $D/sq_field_bw.log; exit 1; }
STAGE=march timeout -k 10 400 bash tools/pmc_sq.sh > $D/sq_march.log 2>&1 || { tail -20 $D/sq_march.log; exit 1; }
ls gpurun_out/pmc_sq_*.txt
# the graph-to-graph gap: the step without the main stream's wait for the march event (1) or without
# the start event (2) -- UNSAFE orderings, measurement only (MFNERF_GAP_TEST, temporary)
for rep in 1 2; do
for G in 0 1 2; do
  MFNERF_GAP_TEST=$G timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > $D/gap_$G.json 2> $D/gap_$G.err || { tail -20 $D/gap_$G.err; exit 1; }
  python -c "import json;d=json.load(open('$D/gap_$G.json'));print('gap$G',d['ms_per_step'])"
done
done
cd /tmp && MFNERF_GAP_TEST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_gap1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof_gap1.log 2>&1 && cd $GRAFT_REPO_ROOT || exit $?
python3 tools/step_timeline.py $D/prof_gap1 > $D/timeline_gap1.txt && tail -4 $D/timeline_gap1.txt

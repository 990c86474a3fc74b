# r5f1: round-5 closing evidence for the final tree, part 1: PMC traffic / MFMA busy (Lego T2^19 and
# T2^20), the bench's kernel stats + step timeline (default and the data-parallel rehearsal).
set -o pipefail
D=gpurun_out/r5f1
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 bash tools/gpu_pmc.sh > $D/pmc.log 2>&1 || { tail -20 $D/pmc.log; exit 1; }
LOG2T=20 timeout -k 10 600 bash tools/gpu_pmc.sh > $D/pmc_T20.log 2>&1 || { tail -20 $D/pmc_T20.log; exit 1; }
ls gpurun_out/pmc_traffic*.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 && cd $GRAFT_REPO_ROOT || exit $?
python3 tools/step_timeline.py $D/prof > $D/timeline.txt && head -1 $D/timeline.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_dp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --dp-rehearse > $GRAFT_REPO_ROOT/$D/prof_dp.log 2>&1 && cd $GRAFT_REPO_ROOT || exit $?
python3 tools/step_timeline.py $D/prof_dp > $D/timeline_dp.txt && head -1 $D/timeline_dp.txt

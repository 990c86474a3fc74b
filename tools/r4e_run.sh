set -o pipefail
D=gpurun_out/r4e
mkdir -p $D
export TMPDIR=/tmp
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
B="timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline"
$B > $D/bench.json 2> $D/bench.err || exit $?
$B --dp-rehearse > $D/bench_dp_direct.json 2> $D/bench_dp_direct.err || exit $?
MFNERF_DIRECT_RCCL=0 $B --dp-rehearse > $D/bench_dp_torch.json 2> $D/bench_dp_torch.err || exit $?
$B --log2-T 20 > $D/bench_T20.json 2> $D/bench_T20.err || exit $?
$B --preset mf128 > $D/bench_mf128.json 2> $D/bench_mf128.err || exit $?
MFNERF_GATE_AT=field_bw $B > $D/bench_gfb.json 2> $D/bench_gfb.err || exit $?
$B > $D/bench2.json 2> $D/bench2.err || exit $?
MFNERF_GATE_AT=field_bw $B > $D/bench_gfb2.json 2> $D/bench_gfb2.err || exit $?
STAGE=grid_bw bash tools/pmc_sq.sh || exit $?
bash tools/gpu_pmc.sh || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_dp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --dp-rehearse > $GRAFT_REPO_ROOT/$D/prof_dp.log 2>&1 && cd $GRAFT_REPO_ROOT && \
python tools/step_timeline.py $D/prof_dp > $D/timeline_dp.txt && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 && cd $GRAFT_REPO_ROOT && \
python tools/step_timeline.py $D/prof > $D/timeline.txt

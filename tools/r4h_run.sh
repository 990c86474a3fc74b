set -o pipefail
D=gpurun_out/r4h
mkdir -p $D
export TMPDIR=/tmp
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_field.py tests/test_gpu_occupancy.py tests/test_gpu_dp_replay.py tests/test_gpu_vren.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1; ok
B="timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline"
for rep in 1 2; do
for V in "rot_occ5 1 1 1 1" "rot_occ5 0 1 1 1" "rot_ws6 1 1 1 1" "rot_occ5 1 0 1 1" "rot_occ5 1 1 0 1" "rot_occ5 1 1 1 0"; do
  set -- $V
  MFNERF_LIB=$PWD/ablibs/$1.so MFNERF_BIN_LANEMAP=$2 MFNERF_SLAB_TAIL=$3 MFNERF_GATE_RIDE=$4 MFNERF_GATE_STREAM=$5 $B > $D/ab.json 2> $D/ab.err || exit $?
  python -c "import json;d=json.load(open('$D/ab.json'));print('$1 lanemap=$2 slab=$3 ride=$4 gstream=$5',d['ms_per_step'],d['grid_bw_ms'])" >> $D/ab.txt
done
done
$B --roofline-every 1000 > $D/bench_re1000.json 2> $D/bench_re1000.err || exit $?
$B > $D/bench_re8.json 2> $D/bench_re8.err || exit $?
timeout -k 10 200 python tools/kbench.py grid_bw > $D/kbench.txt 2>&1 || exit $?
MFNERF_BIN_LANEMAP=0 timeout -k 10 200 python tools/kbench.py grid_bw > $D/kbench_lm0.txt 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 && cd $GRAFT_REPO_ROOT && \
python tools/step_timeline.py $D/prof > $D/timeline.txt

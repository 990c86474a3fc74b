set -o pipefail
D=gpurun_out/r4g
mkdir -p $D
export TMPDIR=/tmp
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_parity_train.py::test_training_psnr_matches_reference > $D/tests.log 2>&1; ok
B="timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline"
for rep in 1 2 3; do
for V in "1 1 1" "0 1 1" "1 0 1" "1 1 0"; do
  set -- $V
  MFNERF_BIN_LANEMAP=$1 MFNERF_SLAB_TAIL=$2 MFNERF_GATE_RIDE=$3 $B > $D/ab.json 2> $D/ab.err || exit $?
  python -c "import json;d=json.load(open('$D/ab.json'));print('lanemap=$1 slab=$2 ride=$3',d['ms_per_step'],d['grid_bw_ms'])" >> $D/ab.txt
done
done
timeout -k 10 200 python tools/kbench.py grid_bw > $D/kbench.txt 2>&1 || exit $?
MFNERF_BIN_LANEMAP=0 timeout -k 10 200 python tools/kbench.py grid_bw > $D/kbench_lm0.txt 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 && cd $GRAFT_REPO_ROOT && \
python tools/step_timeline.py $D/prof > $D/timeline.txt && \
STAGE=grid_bw bash tools/pmc_sq.sh && cp gpurun_out/pmc_sq_grid_bw.txt $D/ && \
timeout -k 10 60 python tools/probe_wait_value.py > $D/probe_wait_value.txt 2>&1

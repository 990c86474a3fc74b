set -o pipefail
D=gpurun_out/r4f
mkdir -p $D
export TMPDIR=/tmp
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_parity_train.py::test_training_psnr_matches_reference > $D/tests.log 2>&1; ok
B="timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline"
for rep in 1 2; do
for L in ablibs/base.so ablibs/slab.so -; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/$L; fi
  $B > $D/ab.json 2> $D/ab.err || exit $?
  python -c "import json;d=json.load(open('$D/ab.json'));print('$L',d['ms_per_step'],d['grid_bw_ms'])" >> $D/ab.txt
done
done
unset MFNERF_LIB
$B --dp-rehearse > $D/bench_dp_direct.json 2> $D/bench_dp_direct.err || exit $?
MFNERF_DIRECT_RCCL=0 $B --dp-rehearse > $D/bench_dp_torch.json 2> $D/bench_dp_torch.err || exit $?
timeout -k 10 200 python tools/kbench.py grid_bw field_bw > $D/kbench.txt 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_dp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --dp-rehearse > $GRAFT_REPO_ROOT/$D/prof_dp.log 2>&1 && cd $GRAFT_REPO_ROOT && \
python tools/step_timeline.py $D/prof_dp > $D/timeline_dp.txt && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 && cd $GRAFT_REPO_ROOT && \
python tools/step_timeline.py $D/prof > $D/timeline.txt

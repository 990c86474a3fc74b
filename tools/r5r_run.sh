# r5r: the MLPs weight-gradient fold riding the accumulate launch (no slab_reduce launch between field_bw and
# the scatter in the one-graph step): engine/optim/train/dp-replay tests (the replayed step bit-identical to
# eager steps), then a bench A/B with the fold in the accumulate (1) or a separate launch (0, a temporary
# MFNERF_FOLD_TEST switch), and one profiled step timeline.
set -o pipefail
D=gpurun_out/r5r
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_optim.py tests/test_gpu_train.py tests/test_gpu_dp_replay.py -q --maxfail=3 --timeout 200 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -60 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for rep in 1 2; do
for F in 1 0; do
  MFNERF_FOLD_TEST=$F timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > $D/b_$F.json 2> $D/b_$F.err || { tail -20 $D/b_$F.err; exit 1; }
  python -c "import json;d=json.load(open('$D/b_$F.json'));print('fold=$F',d['ms_per_step'])"
done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1; cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $D/prof > $D/timeline.txt && cat $D/timeline.txt

# r5m: one-pass W = 128 cooperative field backward -- field / tcnn / configs GPU tests, then the mf128
# bench (eager_stage_ms.field_bw) for this build and the previous commit (var/head: two passes), and a
# kernel trace of the mf128 bench.
set -o pipefail
D=gpurun_out/r5m
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_tcnn.py tests/test_gpu_configs.py tests/test_gpu_train.py -q --maxfail=3 --timeout 200 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -60 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for rep in 1 2; do
for L in - head; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; fi
  timeout -k 10 200 python bench.py --preset mf128 --steps 100 --warmup 20 --no-cpu-baseline > $D/b_$L.json 2> $D/b_$L.err || { tail -20 $D/b_$L.err; exit 1; }
  python -c "import json;d=json.load(open('$D/b_$L.json'));print('$L',d['ms_per_step'],d['eager_stage_ms']['field_bw'])"
done
done
unset MFNERF_LIB
cp $D/b_-.json $D/bench_mf128.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --preset mf128 --steps 30 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1; cd $GRAFT_REPO_ROOT
python3 tools/kstats.py $D/prof field_bw slab_reduce

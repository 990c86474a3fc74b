# r5p: march scan at one wave per SIMD and march_expand within 64 VGPRs, so both fit beside the scatter (adder waves
# add this one) -- correctness (field/configs/engine/golden tests), kernel times under kbench's
# grid_bw_binned and grid_bw_fused for this build and the previous commit (var/head), bench A/B,
# one profiled step timeline.
set -o pipefail
D=gpurun_out/r5p
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_vren.py tests/test_gpu_configs.py tests/test_gpu_engine.py tests/test_gpu_golden.py -q --maxfail=3 --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -60 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for L in - head; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; N=new; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; N=$L; fi
  for S in march; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/ktr_${N}_$S -o run --output-format csv -- python3 tools/kbench.py $S > $D/ktr_${N}_$S.log 2>&1 || { tail -20 $D/ktr_${N}_$S.log; exit 1; }
    echo "== $N $S"; python3 tools/kstats.py $D/ktr_${N}_$S march_
  done
done
unset MFNERF_LIB
LIBS="- mf-nerf_amd/csrc/var/head.so" STEPS=300 TESTS=tests/test_gpu_vren.py bash tools/ab_libs.sh
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1; cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $D/prof > $D/timeline.txt && cat $D/timeline.txt

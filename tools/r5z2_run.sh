# r5z2: the planar forward encode with branch-free gathers (all of a lane's 16 gathers in flight
# before the first use) -- encode / field / configs / engine / golden tests, kbench grid_fw_planar
# new vs var/head (HEAD), bench A/B, timeline.
set -o pipefail
D=gpurun_out/r5z2
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_configs.py tests/test_gpu_engine.py tests/test_gpu_golden.py tests/test_gpu_occupancy.py -q --maxfail=3 --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -60 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for L in - head; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; N=new; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; N=$L; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/ktr_$N -o run --output-format csv -- python3 tools/kbench.py grid_fw_planar > $D/ktr_$N.log 2>&1 || { tail -20 $D/ktr_$N.log; exit 1; }
  echo "== $N"; python3 tools/kstats.py $D/ktr_$N grid_fw
done
unset MFNERF_LIB
LIBS="- mf-nerf_amd/csrc/var/head.so" STEPS=300 TESTS=tests/test_gpu_vren.py bash tools/ab_libs.sh
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1; cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $D/prof > $D/timeline.txt && head -8 $D/timeline.txt

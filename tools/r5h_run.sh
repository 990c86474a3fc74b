# r5h: (1) cheaper march jump search (reciprocal estimate + exact correction) and exact power-of-two
# reciprocals -- bit-exact march tests, march kernel time vs the previous commit (var/head);
# (2) the planar encode's run dedup (var/dedup: every level, var/dedup300: levels with res <= 300) --
# encode tests under each, kbench grid_fw_planar; (3) bench A/B; (4) one profiled step timeline.
set -o pipefail
D=gpurun_out/r5h
mkdir -p $D
export TMPDIR=/tmp
rocprofv3 --list-avail > $D/counters.txt 2>&1 || true
timeout -k 10 500 python -u -m pytest tests/test_gpu_vren.py tests/test_gpu_configs.py tests/test_gpu_engine.py -q --maxfail=5 --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for L in dedup dedup300; do
  MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so timeout -k 10 300 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_golden.py -q -k "planar or encode or golden" --maxfail=3 --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests_$L.log 2>&1 || { tail -30 $D/tests_$L.log; exit 1; }
  echo "$L: $(tail -1 $D/tests_$L.log)"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/ktr_march -o run --output-format csv -- python3 tools/kbench.py march > $D/ktr_march.log 2>&1 && python3 tools/kstats.py $D/ktr_march march_wave
MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/head.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/ktr_march_head -o run --output-format csv -- python3 tools/kbench.py march > $D/ktr_march_head.log 2>&1 && python3 tools/kstats.py $D/ktr_march_head march_wave
for L in - dedup dedup300; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; fi
  echo "== $L"; timeout -k 10 120 python tools/kbench.py grid_fw_planar
done
unset MFNERF_LIB
LIBS="- mf-nerf_amd/csrc/var/head.so mf-nerf_amd/csrc/var/dedup.so mf-nerf_amd/csrc/var/dedup300.so" STEPS=300 TESTS=tests/test_gpu_vren.py bash tools/ab_libs.sh
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1; cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $D/prof > $D/timeline.txt && cat $D/timeline.txt

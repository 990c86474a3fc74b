# r5a: the LDS-DMA accumulate and the two-barrier scatter -- grid/field/engine/config tests, kbench of
# the scatter halves and a bench A/B: round-4 library (var/r4.so), new accumulate only (var/acc.so),
# both (default build).
set -o pipefail
D=gpurun_out/r5a
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_configs.py tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for L in - mf-nerf_amd/csrc/var/acc.so mf-nerf_amd/csrc/var/r4.so; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/$L; fi
  echo "== $L"
  timeout -k 10 200 python tools/kbench.py grid_bw_coarse grid_bw_binned grid_bw grid_bw_fused || exit 1
done
unset MFNERF_LIB
LIBS="- mf-nerf_amd/csrc/var/acc.so mf-nerf_amd/csrc/var/r4.so" STEPS=300 TESTS=tests/test_gpu_vren.py bash tools/ab_libs.sh

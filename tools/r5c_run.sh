# r5c: 16-B LDS-DMA accumulate -- correctness (field/configs/engine tests), per-kernel times under
# kbench's grid_bw_binned for the default build, the 4-B DMA build (var/dma4), probes (1 no adds,
# 2 no DMA, 16 plain record stores) and round 4; then a bench A/B default / plain stores / round 4.
set -o pipefail
D=gpurun_out/r5c
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_configs.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for L in - dma4 probe1 probe2 probe16 r4; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/ktr_$L -o run --output-format csv -- python3 tools/kbench.py grid_bw_binned > $D/ktr_$L.log 2>&1 || { tail -20 $D/ktr_$L.log; exit 1; }
  echo "== $L"; python3 tools/kstats.py $D/ktr_$L bin_scatter bin_accum
done
unset MFNERF_LIB
LIBS="- mf-nerf_amd/csrc/var/probe16.so mf-nerf_amd/csrc/var/r4.so" STEPS=300 TESTS=tests/test_gpu_vren.py bash tools/ab_libs.sh

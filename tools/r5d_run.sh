# r5d: the dense levels as partition records (grid_bw_dense_kernel<NG, true>) -- correctness (field,
# configs, engine, optim, dp, golden), per-kernel times under kbench's grid_bw stages, and a bench A/B
# against the previous commit (var/head.so: dense levels by memory-side atomics), tighter record slots
# (var/s2_32, s2_64: 2 x mean + 32 / 64 records instead of 3 x mean + 96) and round 4.
set -o pipefail
D=gpurun_out/r5d
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_configs.py tests/test_gpu_engine.py tests/test_gpu_optim.py tests/test_gpu_golden.py tests/test_gpu_dp.py -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for L in - head s2_32 s2_64; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/ktr_$L -o run --output-format csv -- python3 tools/kbench.py grid_bw grid_bw_fused > $D/ktr_$L.log 2>&1 || { tail -20 $D/ktr_$L.log; exit 1; }
  echo "== $L"; grep -h "grid_bw" $D/ktr_$L.log; python3 tools/kstats.py $D/ktr_$L grid_bw_dense bin_scatter bin_accum
done
unset MFNERF_LIB
LIBS="- mf-nerf_amd/csrc/var/head.so mf-nerf_amd/csrc/var/s2_32.so mf-nerf_amd/csrc/var/r4.so" STEPS=300 TESTS=tests/test_gpu_vren.py bash tools/ab_libs.sh

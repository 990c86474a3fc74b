# r5e: the accumulate's LDS stage size (records per chunk) -> workgroups per CU: 7936 (default, 2 per CU),
# 3968 (3 per CU, two chunks per Lego partition), 1984 (4 per CU): per-kernel times under kbench and a
# bench A/B.
set -o pipefail
D=gpurun_out/r5e
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_field.py -q -k "binned or partition" --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for L in - rb3968 rb1984; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; fi
  if [ "$L" != "-" ]; then timeout -k 10 300 python -u -m pytest tests/test_gpu_field.py -q -k "binned or partition" --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests_$L.log 2>&1 || { tail -40 $D/tests_$L.log; exit 1; }; tail -1 $D/tests_$L.log; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/ktr_$L -o run --output-format csv -- python3 tools/kbench.py grid_bw grid_bw_fused > $D/ktr_$L.log 2>&1 || { tail -20 $D/ktr_$L.log; exit 1; }
  echo "== $L"; grep -h "grid_bw" $D/ktr_$L.log; python3 tools/kstats.py $D/ktr_$L grid_bw_dense bin_scatter bin_accum
done
unset MFNERF_LIB
LIBS="- mf-nerf_amd/csrc/var/rb3968.so mf-nerf_amd/csrc/var/rb1984.so" STEPS=300 TESTS=tests/test_gpu_vren.py bash tools/ab_libs.sh

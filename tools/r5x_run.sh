# r5x: the accumulate's LDS stage size with the partitioned tables' Adam fused in (the bench's normal
# step): 7936 records (2 workgroups per CU, head) vs 3840 (3 per CU) vs 2560 -- kbench grid_bw_fused and
# the bench A/B.
set -o pipefail
D=gpurun_out/r5x
mkdir -p $D
export TMPDIR=/tmp
for L in head acc3840 acc2560; do
  export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/ktr_$L -o run --output-format csv -- python3 tools/kbench.py grid_bw_fused grid_bw > $D/ktr_$L.log 2>&1 || { tail -20 $D/ktr_$L.log; exit 1; }
  echo "== $L"; python3 tools/kstats.py $D/ktr_$L bin_
done
unset MFNERF_LIB
LIBS="mf-nerf_amd/csrc/var/head.so mf-nerf_amd/csrc/var/acc3840.so mf-nerf_amd/csrc/var/acc2560.so" STEPS=300 TESTS=tests/test_gpu_vren.py bash tools/ab_libs.sh

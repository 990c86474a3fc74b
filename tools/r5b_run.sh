# r5b: where the scatter and the accumulate spend their time -- timing-probe builds (MFN_PROBE bits:
# 1 accumulate without adds, 2 without record DMA, 4 scatter without record stores, 8 without counting
# atomics; results invalid) under a kernel trace of kbench's grid_bw_binned stage; then the march's
# bit-exact tests and a kbench of the march (chunk prefetch).
set -o pipefail
D=gpurun_out/r5b
mkdir -p $D
export TMPDIR=/tmp
for L in - probe1 probe2 probe3 probe4 probe8 probe12; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/ktr_$L -o run --output-format csv -- python3 tools/kbench.py grid_bw_binned > $D/ktr_$L.log 2>&1 || { tail -20 $D/ktr_$L.log; exit 1; }
  echo "== $L"; python3 tools/kstats.py $D/ktr_$L bin_scatter bin_accum
done
unset MFNERF_LIB
timeout -k 10 300 python -u -m pytest tests/test_gpu_vren.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $D/vren.log 2>&1 || { tail -30 $D/vren.log; exit 1; }
tail -1 $D/vren.log
timeout -k 10 200 python tools/kbench.py march > $D/kbench_march.log 2>&1 && cat $D/kbench_march.log
MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/r4.so timeout -k 10 200 python tools/kbench.py march > $D/kbench_march_r4.log 2>&1 && cat $D/kbench_march_r4.log

# r5g1: the MixedFeature preset's scatter (single records, 12 binned levels) with its level loop
# written out like the pair layout's -- kbench grid_bw on the mf128 preset, new vs var/head; configs
# tests (MixedFeature scatter parity) first.
set -o pipefail
D=gpurun_out/r5g1
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_field.py -q --maxfail=3 --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -60 $D/tests.log; exit 1; }
tail -1 $D/tests.log
export MFNERF_KBENCH_PRESET=mf128
for L in - head; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; N=new; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; N=$L; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $D/ktr_$N -o run --output-format csv -- python3 tools/kbench.py grid_bw > $D/ktr_$N.log 2>&1 || { tail -20 $D/ktr_$N.log; exit 1; }
  echo "== $N"; python3 tools/kstats.py $D/ktr_$N bin_ dense
done
unset MFNERF_LIB MFNERF_KBENCH_PRESET
for L in - head; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --preset mf128 > $D/b_$L.json 2> $D/b_$L.err || { tail -20 $D/b_$L.err; exit 1; }
  python -c "import json;d=json.load(open('$D/b_$L.json'));print('$L',d['ms_per_step'],d.get('grid_bw_ms'))"
done

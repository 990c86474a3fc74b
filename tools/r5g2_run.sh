# r5g2: MixedFeature x-pairs as pair records where the canonical step is 1 or 2 (shift bit in the
# record) -- configs / field / engine tests, kbench grid_bw on the mf128 preset new vs var/head, the
# mf128 bench A/B, and the Lego bench (pair layout, unchanged path) once.
set -o pipefail
D=gpurun_out/r5g2
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_field.py tests/test_gpu_engine.py -q --maxfail=3 --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -60 $D/tests.log; exit 1; }
tail -1 $D/tests.log
export MFNERF_KBENCH_PRESET=mf128
for L in - head; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; N=new; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; N=$L; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $D/ktr_$N -o run --output-format csv -- python3 tools/kbench.py grid_bw > $D/ktr_$N.log 2>&1 || { tail -20 $D/ktr_$N.log; exit 1; }
  echo "== $N"; python3 tools/kstats.py $D/ktr_$N bin_ dense
done
unset MFNERF_LIB MFNERF_KBENCH_PRESET
for r in 1 2; do
for L in - head; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --preset mf128 > $D/b_$L.json 2> $D/b_$L.err || { tail -20 $D/b_$L.err; exit 1; }
  python -c "import json;d=json.load(open('$D/b_$L.json'));print('$L',d['ms_per_step'],d.get('grid_bw_ms'))"
done
done
unset MFNERF_LIB
timeout -k 10 200 python bench.py --no-cpu-baseline > $D/b_lego.json 2> $D/b_lego.err || { tail -20 $D/b_lego.err; exit 1; }
python -c "import json;d=json.load(open('$D/b_lego.json'));print('lego',d['ms_per_step'],d.get('grid_bw_ms'))"

# r5g7: the fused accumulate's optimizer state (p, m, v) loaded and stored non-temporally -- optim /
# engine tests, bench A/B (Lego and mf128) vs var/head.
set -o pipefail
D=gpurun_out/r5g7
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_engine.py -q --maxfail=3 --timeout 300 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -60 $D/tests.log; exit 1; }
tail -1 $D/tests.log
LIBS="- mf-nerf_amd/csrc/var/head.so" STEPS=300 TESTS=tests/test_gpu_vren.py bash tools/ab_libs.sh
LIBS="- mf-nerf_amd/csrc/var/head.so" STEPS=300 TESTS=tests/test_gpu_vren.py bash tools/ab_libs.sh
for L in - head; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --preset mf128 > $D/b_$L.json 2> $D/b_$L.err || { tail -20 $D/b_$L.err; exit 1; }
  python -c "import json;d=json.load(open('$D/b_$L.json'));print('mf128 $L',d['ms_per_step'],d.get('grid_bw_ms'))"
done

# r5g3: the scatter's LDS cursors for 5120 partitions (every partition of the Lego layout at T 2^20)
# -- engine / configs tests, the T 2^20 and T 2^19 bench A/B vs var/head.
set -o pipefail
D=gpurun_out/r5g3
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_configs.py -q --maxfail=3 --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -60 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for r in 1 2; do
for L in - head; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --log2-T 20 --steps 300 > $D/t20_$L.json 2> $D/t20_$L.err || { tail -20 $D/t20_$L.err; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 > $D/t19_$L.json 2> $D/t19_$L.err || { tail -20 $D/t19_$L.err; exit 1; }
  python -c "import json;a=json.load(open('$D/t20_$L.json'));b=json.load(open('$D/t19_$L.json'));print('$L','T20',a['ms_per_step'],a.get('grid_bw_ms'),'T19',b['ms_per_step'],b.get('grid_bw_ms'))"
done
done

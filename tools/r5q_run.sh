# r5q: occupancy probes in row-major cell order (hashed levels' x-neighbours share table lines in the
# refresh's encode) -- occupancy tests, then density_update_ms of the bench for this build and the
# previous commit (var/head), plus a kernel trace of the refresh.
set -o pipefail
D=gpurun_out/r5q
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_occupancy.py tests/test_gpu_engine.py -q --maxfail=3 --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -60 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for rep in 1 2; do
for L in - head; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; fi
  timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > $D/b_$L.json 2> $D/b_$L.err || { tail -20 $D/b_$L.err; exit 1; }
  python -c "import json;d=json.load(open('$D/b_$L.json'));print('$L',d['ms_per_step'],d['density_update_ms'])"
done
done

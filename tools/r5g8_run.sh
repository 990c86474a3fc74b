# r5g8: the optimizer-state streams of the Adam kernels (adam.hip, adam_fixed_body) non-temporal too
# -- optim / dp / engine tests, the Lego and DP-rehearsal bench A/B vs var/head.
set -o pipefail
D=gpurun_out/r5g8
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_engine.py tests/test_gpu_dp.py tests/test_gpu_dp_replay.py -q --maxfail=3 --timeout 300 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -60 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for r in 1 2; do
for L in - head; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 > $D/b_$L.json 2> $D/b_$L.err || { tail -20 $D/b_$L.err; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 --dp-rehearse > $D/d_$L.json 2> $D/d_$L.err || { tail -20 $D/d_$L.err; exit 1; }
  python -c "import json;a=json.load(open('$D/b_$L.json'));b=json.load(open('$D/d_$L.json'));print('$L','N1',a['ms_per_step'],'DP',b['ms_per_step'])"
done
done

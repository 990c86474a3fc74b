# r5g9: the accumulate's record DMA loads non-temporal (records are read once) -- the full GPU suite
# + smoke, then the bench A/B vs var/head (HEAD).
set -o pipefail
D=gpurun_out/r5g9
mkdir -p $D
export TMPDIR=/tmp
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1; ok
tail -1 $D/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
tail -1 $D/smoke.log
for r in 1 2; do
for L in - head; do
  if [ "$L" = "-" ]; then unset MFNERF_LIB; else export MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/$L.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 > $D/b_$L.json 2> $D/b_$L.err || { tail -20 $D/b_$L.err; exit 1; }
  python -c "import json;a=json.load(open('$D/b_$L.json'));print('$L',a['ms_per_step'],a.get('grid_bw_ms'))"
done
done
unset MFNERF_LIB
timeout -k 10 300 python bench.py > $D/bench.json 2> $D/bench.err || exit $?
python -c "import json;d=json.load(open('$D/bench.json'));print('bench',d['ms_per_step'],d['value'],d.get('grid_bw_ms'),d['roofline']['frac'])"

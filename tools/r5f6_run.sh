# r5f6: closing evidence of the final tree (after the non-temporal Adam kernels): the full GPU suite + smoke and
# the default bench line with the CPU baseline, the data-parallel rehearsal, the mf128 line.
set -o pipefail
D=gpurun_out/r5f6
mkdir -p $D
export TMPDIR=/tmp
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1; ok
tail -1 $D/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
tail -1 $D/smoke.log
timeout -k 10 300 python bench.py > $D/bench.json 2> $D/bench.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --preset mf128 > $D/bench_mf128.json 2> $D/bench_mf128.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --dp-rehearse > $D/bench_dp_rehearse.json 2> $D/bench_dp_rehearse.err || exit $?
for f in bench bench_mf128 bench_dp_rehearse; do python -c "import json;d=json.load(open('$D/$f.json'));print('$f',d['ms_per_step'],d['value'],d.get('grid_bw_ms'),d.get('density_update_ms'),d['roofline']['frac'])"; done

# r5f2: round-5 closing evidence for the final tree, part 2: the full GPU suite (parity protocol
# included) + smoke, the bench lines (default with the CPU baseline, mf128, T2^20, the data-parallel
# rehearsal), the mf128 PMC traffic, the 30k-step protocol and the render FPS.
set -o pipefail
D=gpurun_out/r5f2
mkdir -p $D
export TMPDIR=/tmp
export MFNERF_PARITY_OUT=$GRAFT_REPO_ROOT/$D/parity_train.json
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1; ok
tail -1 $D/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
tail -1 $D/smoke.log
PRESET=mf128 timeout -k 10 500 bash tools/gpu_pmc.sh > $D/pmc_mf128.log 2>&1 || { tail -20 $D/pmc_mf128.log; exit 1; }
cp gpurun_out/pmc_traffic_mf128.json profiles/r05_v24_pmc_traffic_mf128.json
timeout -k 10 300 python bench.py > $D/bench.json 2> $D/bench.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --preset mf128 > $D/bench_mf128.json 2> $D/bench_mf128.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --log2-T 20 > $D/bench_T20.json 2> $D/bench_T20.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --dp-rehearse > $D/bench_dp_rehearse.json 2> $D/bench_dp_rehearse.err || exit $?
for f in bench bench_mf128 bench_T20 bench_dp_rehearse; do python -c "import json;d=json.load(open('$D/$f.json'));print('$f',d['ms_per_step'],d['value'],d.get('grid_bw_ms'),d.get('density_update_ms'),d['roofline']['frac'],d['roofline'].get('traffic'))"; done
timeout -k 10 400 python tools/train_30k.py > $D/train30k.json 2> $D/train30k.err || exit $?
tail -c 300 $D/train30k.json
timeout -k 10 300 python tools/render_fps.py > $D/render_fps.json 2> $D/render_fps.err || { tail -20 $D/render_fps.err; exit 1; }
cat $D/render_fps.json

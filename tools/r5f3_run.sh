# r5f3: closing evidence after the MixedFeature pair records: the full GPU suite + smoke, PMC traffic
# (Lego T2^19 and mf128), the bench lines (default with the CPU baseline, mf128, T2^20, DP rehearsal),
# the step timeline.
set -o pipefail
D=gpurun_out/r5f3
mkdir -p $D
export TMPDIR=/tmp
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1; ok
tail -1 $D/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
tail -1 $D/smoke.log
timeout -k 10 600 bash tools/gpu_pmc.sh > $D/pmc.log 2>&1 || { tail -20 $D/pmc.log; exit 1; }
PRESET=mf128 timeout -k 10 600 bash tools/gpu_pmc.sh > $D/pmc_mf128.log 2>&1 || { tail -20 $D/pmc_mf128.log; exit 1; }
cp gpurun_out/pmc_traffic.json profiles/r05_v28_pmc_traffic.json
cp gpurun_out/pmc_traffic_mf128.json profiles/r05_v28_pmc_traffic_mf128.json
timeout -k 10 300 python bench.py > $D/bench.json 2> $D/bench.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --preset mf128 > $D/bench_mf128.json 2> $D/bench_mf128.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --log2-T 20 > $D/bench_T20.json 2> $D/bench_T20.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --dp-rehearse > $D/bench_dp_rehearse.json 2> $D/bench_dp_rehearse.err || exit $?
for f in bench bench_mf128 bench_T20 bench_dp_rehearse; do python -c "import json;d=json.load(open('$D/$f.json'));print('$f',d['ms_per_step'],d['value'],d.get('grid_bw_ms'),d.get('density_update_ms'),d['roofline']['frac'],d['roofline'].get('traffic'))"; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 && cd $GRAFT_REPO_ROOT || exit $?
python3 tools/step_timeline.py $D/prof > $D/timeline.txt && head -1 $D/timeline.txt

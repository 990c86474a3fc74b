# Occupancy refresh fusions: occupancy tests, poisoned-buffer diagnostic, bench (density_update_ms), kernel stats.
set -o pipefail
D=gpurun_out/r4aa
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_occupancy.py tests/test_gpu_engine.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || exit $?
timeout -k 10 120 python tools/diag_occ.py --poison > $D/diag.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $D/bench.json 2> $D/bench.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 && cd $GRAFT_REPO_ROOT || exit $?

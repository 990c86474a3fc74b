# r5g6: the gate's atomics relaxed (placement only): the polling wave's agent-scope acquire invalidated
# one XCD's L2 every ~0.2 us through the chain, and the signal's release wrote an XCD's L2 back --
# engine / vren / dp_replay tests, bench A/B vs var/head (HEAD), step timeline.
set -o pipefail
D=gpurun_out/r5g6
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_dp_replay.py tests/test_gpu_train.py -q --maxfail=3 --timeout 300 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -60 $D/tests.log; exit 1; }
tail -1 $D/tests.log
LIBS="- mf-nerf_amd/csrc/var/head.so" STEPS=300 TESTS=tests/test_gpu_vren.py bash tools/ab_libs.sh
LIBS="- mf-nerf_amd/csrc/var/head.so" STEPS=300 TESTS=tests/test_gpu_vren.py bash tools/ab_libs.sh
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1; cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $D/prof > $D/timeline.txt && cat $D/timeline.txt

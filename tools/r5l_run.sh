# r5l: the full GPU suite (parity protocol included: MFNERF_PARITY_OUT) and smoke on the current tree.
set -o pipefail
D=gpurun_out/r5l
mkdir -p $D
export TMPDIR=/tmp
export MFNERF_PARITY_OUT=$GRAFT_REPO_ROOT/$D/parity_train.json
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1; ok
tail -3 $D/tests.log
grep -E "FAILED|ERROR" $D/tests.log | head -20; ok
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
tail -2 $D/smoke.log

#!/bin/bash
# GPU session: selected tests, then a rocprofv3 kernel-stats profile of a short bench run.
#   TESTS="tests/test_gpu_field.py" OUT=prof bash tools/gpu_prof.sh
set -o pipefail
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
OUT=${OUT:-prof}
timeout -k 10 600 python -m pytest $TESTS -m gpu -x -q -p no:cacheprovider > gpurun_out/t.log 2>&1
rc=$?
tail -2 gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$OUT -o run --output-format csv -- python3 bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline > gpurun_out/$OUT.log 2>&1
rc=$?
grep '"metric"' gpurun_out/$OUT.log | cut -c1-400
exit $rc

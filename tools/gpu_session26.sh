#!/bin/bash
# Mixed timed/fused replays vs eager (bit-identical), then the whole GPU suite once more.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/s26_tests.log 2>&1
rc=$?
echo "EXIT $rc"; grep -E "passed|failed|Error" gpurun_out/s26_tests.log | tail -5
exit $rc

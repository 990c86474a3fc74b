#!/bin/bash
# Side-stream march placement/priority sweep: (late, high) default, (early, normal), (late, normal).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s25_late_hi.json 2> gpurun_out/s25_a.err && \
MFNERF_MARCH_EARLY=1 MFNERF_SIDE_HIGH_PRIORITY=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s25_early_lo.json 2> gpurun_out/s25_b.err && \
MFNERF_SIDE_HIGH_PRIORITY=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s25_late_lo.json 2> gpurun_out/s25_c.err
rc=$?
echo "EXIT $rc"; for f in late_hi early_lo late_lo; do echo $f; cut -c100-190 gpurun_out/s25_$f.json; done
exit $rc

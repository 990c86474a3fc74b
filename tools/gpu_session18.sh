#!/bin/bash
# The reference's 30k-step training protocol on the textured and flat ball scenes: wall time + test PSNR.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/train_30k.py --tex 40 > gpurun_out/s18_train30k_tex.log 2>&1 && \
timeout -k 10 400 python -u tools/train_30k.py --tex 0 > gpurun_out/s18_train30k_flat.log 2>&1
rc=$?
echo "EXIT $rc"; tail -n 4 gpurun_out/s18_train30k_tex.log | cut -c1-400; tail -n 2 gpurun_out/s18_train30k_flat.log | cut -c1-400
exit $rc

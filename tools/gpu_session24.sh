#!/bin/bash
# Whole training protocols on the round-end tree: Lego defaults (30k x 8192, Hash T19) and the MF
# benchmark schedule (20k x 16384, MixedFeature 8 tables T20, rgb 128), textured ball scene.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/train_30k.py --tex 40 > gpurun_out/s24_train_hash.log 2>&1 && \
timeout -k 10 500 python -u tools/train_30k.py --tex 40 --mf > gpurun_out/s24_train_mf.log 2>&1
rc=$?
echo "EXIT $rc"; tail -n 1 gpurun_out/s24_train_hash.log | cut -c1-420; tail -n 1 gpurun_out/s24_train_mf.log | cut -c1-420
exit $rc

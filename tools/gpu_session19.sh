#!/bin/bash
# PMC refresh on the current tree: HBM-side bytes per launch (FETCH_SIZE / WRITE_SIZE, separate
# passes) and MFMA busy cycles, each pass its own short bench run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/s19_fetch -o pmc --output-format csv -- $B > gpurun_out/s19_fetch.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/s19_write -o pmc --output-format csv -- $B > gpurun_out/s19_write.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES -d gpurun_out/s19_mfma -o pmc --output-format csv -- $B > gpurun_out/s19_mfma.log 2>&1
rc=$?
echo "EXIT $rc"
python3 tools/pmc_traffic.py gpurun_out/s19_fetch gpurun_out/s19_write > gpurun_out/s19_pmc_traffic.json; head -c 1500 gpurun_out/s19_pmc_traffic.json
exit $rc

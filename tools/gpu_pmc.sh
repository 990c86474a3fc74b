#!/bin/bash
# Round-end profiles (GPU): kernel stats of a bench run, then the PMC passes (one counter group per
# rocprofv3 run, MI355X_MICROARCH.md): FETCH_SIZE, WRITE_SIZE, TCC_EA0_ATOMIC_sum, MFMA busy.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --roofline-every 1"  # every scatter launch unfused, as the timed ones
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- $B > gpurun_out/prof.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $B > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- $B > gpurun_out/pmc_write.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d gpurun_out/pmc_atomic -o run --output-format csv -- $B > gpurun_out/pmc_atomic.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mfma -o run --output-format csv -- $B > gpurun_out/pmc_mfma.log 2>&1
rc=$?
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_atomic > gpurun_out/pmc_traffic.json
python tools/pmc_summary.py gpurun_out/pmc_mfma > gpurun_out/pmc_mfma.txt
exit $rc

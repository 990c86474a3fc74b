#!/bin/bash
# Round-end profiles (GPU): kernel stats of a bench run, then the PMC passes (one counter group per
# rocprofv3 run, MI355X_MICROARCH.md): FETCH_SIZE, WRITE_SIZE, TCC_EA0_ATOMIC_sum, MFMA busy.
# PRESET=mf128 profiles the MixedFeature / rgb-128 preset (outputs suffixed _mf128); LOG2T=20 another
# table size (suffix _T20: bench.py pmc_suffix keys the summaries on the workload).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${PRESET:-lego}
X=$(python3 -c "import bench; print(bench.pmc_suffix('$P', ${LOG2T:-None}, None))")
B="python3 bench.py --preset $P ${LOG2T:+--log2-T $LOG2T} --steps 20 --warmup 5 --no-cpu-baseline --roofline-every 1"  # every scatter launch unfused, as the timed ones
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof$X -o run --output-format csv -- $B > gpurun_out/prof$X.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch$X -o run --output-format csv -- $B > gpurun_out/pmc_fetch$X.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write$X -o run --output-format csv -- $B > gpurun_out/pmc_write$X.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d gpurun_out/pmc_atomic$X -o run --output-format csv -- $B > gpurun_out/pmc_atomic$X.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mfma$X -o run --output-format csv -- $B > gpurun_out/pmc_mfma$X.log 2>&1
rc=$?
python tools/pmc_traffic.py gpurun_out/pmc_fetch$X gpurun_out/pmc_write$X gpurun_out/pmc_atomic$X > gpurun_out/pmc_traffic$X.json
python tools/pmc_summary.py gpurun_out/pmc_mfma$X > gpurun_out/pmc_mfma$X.txt
exit $rc

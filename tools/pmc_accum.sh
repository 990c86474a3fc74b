#!/bin/bash
# One SQ counter pass over a short bench (the partitioned accumulate's issue profile).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --roofline-every 1"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/pmc_sq1 -o run --output-format csv -- $B > gpurun_out/pmc_sq1.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq2 -o run --output-format csv -- $B > gpurun_out/pmc_sq2.log 2>&1
rc=$?
python tools/pmc_summary.py gpurun_out/pmc_sq1 > gpurun_out/pmc_sq1.txt
python tools/pmc_summary.py gpurun_out/pmc_sq2 > gpurun_out/pmc_sq2.txt
exit $rc

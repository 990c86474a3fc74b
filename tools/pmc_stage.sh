#!/bin/bash
# kernel trace + PMC passes over one kbench stage (GPU): STAGE=grid_bw_coarse KSUB=dense bash tools/pmc_stage.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${STAGE:-grid_bw_coarse}
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ktr -o run --output-format csv -- python3 tools/kbench.py $STAGE > gpurun_out/ktr.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc1 -o run --output-format csv -- python3 tools/kbench.py $STAGE > gpurun_out/pmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_SALU TCC_EA0_ATOMIC_sum -d gpurun_out/pmc2 -o run --output-format csv -- python3 tools/kbench.py $STAGE > gpurun_out/pmc2.log 2>&1
rc=$?
grep -i "${KSUB:-dense}" gpurun_out/ktr/run_kernel_stats.csv | cut -c1-200
for d in pmc1 pmc2; do python tools/pmc_summary.py gpurun_out/$d ${KSUB:-dense}; done
exit $rc

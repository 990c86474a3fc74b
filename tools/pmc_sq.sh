#!/bin/bash
# Issue profile of one kbench stage (GPU box): a kernel trace and three SQ counter passes, each its
# own rocprofv3 run, summarised per kernel (median per dispatch) into gpurun_out/pmc_sq_<stage>.txt.
#     STAGE=grid_bw bash tools/pmc_sq.sh
# tools/pmc_sq_report.py derives the shares of the waves' resident cycles (waiting, issue-blocked,
# issuing VALU / LDS), LDS conflict cycles per active LDS cycle and the average VMEM reads in flight.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${STAGE:-grid_bw}
O=gpurun_out/pmc_sq_$STAGE
rm -rf $O && mkdir -p $O
K="python3 tools/kbench.py $STAGE"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/ktr -o run --output-format csv -- $K > $O/ktr.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/p1 -o run --output-format csv -- $K > $O/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_ANY -d $O/p2 -o run --output-format csv -- $K > $O/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN -d $O/p3 -o run --output-format csv -- $K > $O/p3.log 2>&1
rc=$?
python3 tools/pmc_sq_report.py $O > gpurun_out/pmc_sq_$STAGE.txt 2>&1
exit $rc

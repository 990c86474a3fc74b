# r5s: L2 (TCC) counters of the partitioned scatter and accumulate (kbench grid_bw_binned, eager, 27
# launches): hits / misses / memory-side read requests (all, DRAM), read-request latency, tag and
# DRAM-credit stalls -- where the accumulate's ~3 TB/s record loads wait.
set -o pipefail
D=gpurun_out/r5s
mkdir -p $D
export TMPDIR=/tmp
K="python3 tools/kbench.py grid_bw_binned"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d $D/pa -o run --output-format csv -- $K > $D/pa.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_READ_sum TCC_READ_REQ_LATENCY_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum -d $D/pb -o run --output-format csv -- $K > $D/pb.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum TCC_BUSY_sum -d $D/pc -o run --output-format csv -- $K > $D/pc.log 2>&1
rc=$?
python3 tools/pmc_summary.py $D/pa > $D/pa.txt 2>&1; python3 tools/pmc_summary.py $D/pb > $D/pb.txt 2>&1; python3 tools/pmc_summary.py $D/pc > $D/pc.txt 2>&1
grep -A6 "bin_accum\|bin_scatter" $D/pa.txt $D/pb.txt $D/pc.txt | head -60
exit $rc

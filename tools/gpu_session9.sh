#!/bin/bash
# Counters of the compositing kernels (one PMC pass) + their per-stage timings.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/kbench.py composite composite_fw composite_bw > gpurun_out/s9_kb.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH -d gpurun_out/s9_pmc -o pmc --output-format csv -- python3 tools/kbench.py composite > gpurun_out/s9_pmc.log 2>&1
rc=$?
echo "EXIT $rc"; tail -4 gpurun_out/s9_kb.log
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/s9_pmc/**/*counter_collection.csv", recursive=True)
print(f)
if f:
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"][:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
    for k, d in acc.items():
        if "composite" in k:
            n = cnt[(k, "SQ_WAVES")]
            print(k, n, {c: round(v / max(n, 1)) for c, v in d.items()})
PY
exit $rc

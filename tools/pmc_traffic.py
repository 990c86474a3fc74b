"""Per-launch HBM-side traffic of each kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE),
corrected as /opt/skills/guides/MI355X_MICROARCH.md prescribes for gfx950: counters are in KiB,
FETCH_SIZE reports half the bytes of wide coalesced streaming reads (doubled here; grid_bw's reads
are such streams: dL/dy rows and positions), WRITE_SIZE is exact for float atomics.

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write [gpurun_out/pmc_atomic] \
        > profiles/rNN_pmc_traffic.json

The optional third pass (TCC_EA0_ATOMIC_sum) adds each kernel's memory-side atomic requests per
launch (every float/int global atomic leaves L2 as one request per 64-B segment, MI355X_MICROARCH.md
'Global float atomics'), the quantity the table-gradient scatter is bound by.
"""
import collections
import csv
import glob
import json
import sys


def per_launch(d, counter):
    f = sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True))[0]
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sorted(v)[len(v) // 2] * 1024.0 for k, v in vals.items()}  # median launch, bytes


def per_launch_raw(d, counter):
    f = sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True))[0]
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sorted(v)[len(v) // 2] for k, v in vals.items()}


fetch, write = per_launch(sys.argv[1], "FETCH_SIZE"), per_launch(sys.argv[2], "WRITE_SIZE")
atomic = per_launch_raw(sys.argv[3], "TCC_EA0_ATOMIC_sum") if len(sys.argv) > 3 else {}
out = {}
for k in sorted(set(fetch) & set(write), key=lambda k: -(fetch[k] + write[k])):
    short = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    out[short] = {"fetch_bytes_corrected": 2 * fetch[k], "write_bytes": write[k],
                  "traffic_bytes": 2 * fetch[k] + write[k]}
    if k in atomic:
        out[short]["atomic_requests"] = atomic[k]
json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE" + (" / --pmc TCC_EA0_ATOMIC_sum" if atomic else "")
                     + " (separate passes) --kernel-trace, "
                     "python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline; median launch",
           "kernels": out}, sys.stdout, indent=1)
print()

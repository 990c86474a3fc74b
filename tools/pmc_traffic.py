"""Per-launch HBM-side traffic of each kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE),
corrected as /opt/skills/guides/MI355X_MICROARCH.md prescribes for gfx950: counters are in KiB,
FETCH_SIZE reports half the bytes of wide coalesced streaming reads (doubled here; grid_bw's reads
are such streams: dL/dy rows and positions), WRITE_SIZE is exact for float atomics.

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/rNN_pmc_traffic.json
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


fetch, write = per_launch(sys.argv[1], "FETCH_SIZE"), per_launch(sys.argv[2], "WRITE_SIZE")
out = {}
for k in sorted(set(fetch) & set(write), key=lambda k: -(fetch[k] + write[k])):
    short = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    out[short] = {"fetch_bytes_corrected": 2 * fetch[k], "write_bytes": write[k],
                  "traffic_bytes": 2 * fetch[k] + write[k]}
json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) --kernel-trace, "
                     "python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline; median launch",
           "kernels": out}, sys.stdout, indent=1)
print()

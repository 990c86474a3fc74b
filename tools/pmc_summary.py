"""Median per-dispatch PMC values per kernel from a rocprofv3 counter_collection.csv.
    python tools/pmc_summary.py <dir-or-csv> [kernel-substring]"""
import collections
import csv
import glob
import os
import sys

path = sys.argv[1]
if os.path.isdir(path):
    path = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)[0]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(path)):
    if sub in r["Kernel_Name"]:
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        v = sorted(v)
        print(f"   {c:28s} n={len(v):3d} median={v[len(v) // 2]:.5g}")

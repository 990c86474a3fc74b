"""Print name / calls / average us of the kernels matching a pattern from rocprofv3 --stats output
(the *kernel_stats.csv under DIR).    python tools/kstats.py DIR [pattern ...]"""
import csv
import glob
import os
import sys

d, pats = sys.argv[1], sys.argv[2:]
for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row["Name"]
        if not pats or any(p in name for p in pats):
            print(f"{name[:60]:60s} calls {int(row['Calls']):5d}  avg {float(row['AverageNs']) / 1e3:8.1f} us  "
                  f"min {float(row['MinNs']) / 1e3:8.1f}")

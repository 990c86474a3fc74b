"""Print the top kernels of a rocprofv3 kernel-stats CSV:  python tools/prof_summary.py gpurun_out/prof [N]"""
import csv
import glob
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
f = sorted(glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True))[0]
for x in list(csv.DictReader(open(f)))[:n]:
    print(f"{x['Calls']:>5} {float(x['TotalDurationNs']) / 1e6:9.3f} ms  avg {float(x['AverageNs']) / 1e3:8.1f} us"
          f"  max {float(x['MaxNs']) / 1e3:8.1f} us  {x['Name'][:90]}")

"""One graph-replayed training step's kernel timeline from a rocprofv3 --kernel-trace CSV:
start/end (us, relative to the step's grid_bw start) and queue of every kernel between two
consecutive grid_bw launches near the end of the run.

    python tools/step_timeline.py gpurun_out/prof/run_kernel_trace.csv
"""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
    gb = [k for k in ks if "grid_bw_kernel" in k[2]]
    a, b = gb[-3][0], gb[-2][0]
    t0 = a
    print(f"step (grid_bw start to next grid_bw start): {(b - a) / 1e3:.1f} us")
    for s, e, n, q in ks:
        if a <= s < b:
            print(f"{(s - t0) / 1e3:8.1f} - {(e - t0) / 1e3:8.1f}  q{q}  {n[:90]}")


if __name__ == "__main__":
    main(sys.argv[1])

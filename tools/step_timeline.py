"""One training step's kernel timeline from a rocprofv3 --kernel-trace CSV of a bench run: the
kernels between the starts of two consecutive launches of an anchor kernel (default: the chain's
first kernel on the main queue, grid_fw_planar), in start order, with queue ids, relative to the
step start.  Picks the median-length step of the last `--last` replayed steps.

    python tools/step_timeline.py gpurun_out/prof [--anchor grid_fw_planar] [--last 20]
"""
import argparse
import csv
import glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--anchor", default="grid_fw_planar")
    ap.add_argument("--last", type=int, default=20)
    a = ap.parse_args()
    f = sorted(glob.glob(a.dir + "/**/*kernel_trace.csv", recursive=True))[0]
    rows = []
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), name))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[3].startswith(a.anchor)]
    steps = [(rows[starts[k + 1]][0] - rows[starts[k]][0], starts[k], starts[k + 1])
             for k in range(max(0, len(starts) - 1 - a.last), len(starts) - 1)]
    steps.sort()
    dt, i0, i1 = steps[len(steps) // 2]
    t0 = rows[i0][0]
    print(f"step ({a.anchor} start to next {a.anchor} start): {dt / 1e3:.1f} us (median of {len(steps)})")
    for s, e, q, n in rows[i0:i1]:
        print(f"{(s - t0) / 1e3:8.1f} - {(e - t0) / 1e3:8.1f}  q{q}  {n[:90]}")


if __name__ == "__main__":
    main()

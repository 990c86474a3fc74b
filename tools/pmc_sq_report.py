"""Per-kernel summary of tools/pmc_sq.sh's passes: median per dispatch of every SQ counter, plus
the ratios used in DESIGN.md (shares of the waves' resident cycles).
    python tools/pmc_sq_report.py gpurun_out/pmc_sq_<stage> [kernel-substring]"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    """The kernel's own name (template arguments kept, namespace and parameter list dropped)."""
    m = re.search(r"(\w+)(<[^()]*>)?\(", name.replace("(anonymous namespace)::", ""))
    return m.group(1) + (m.group(2) or "") if m else name[:70]


root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"]:
            vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
med = {k: {c: sorted(v)[len(v) // 2] for c, v in d.items()} for k, d in vals.items()}
ratios = [("waiting (any)", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"),
          ("issue-blocked", "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"),
          ("issuing VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES"),
          ("issuing LDS", "SQ_ACTIVE_INST_LDS", "SQ_WAVE_CYCLES"),
          ("issuing any", "SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES"),
          ("LDS wait (inst)", "SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES"),
          ("LDS bank conflict / LDS active", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"),
          ("LDS address conflict / LDS active", "SQ_LDS_ADDR_CONFLICT", "SQ_LDS_IDX_ACTIVE"),
          ("LDS active cycles per LDS instr", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_LDS"),
          ("VMEM reads in flight (avg)", "SQ_INST_LEVEL_VMEM", "SQ_WAVE_CYCLES"),
          ("waves resident per busy cycle", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES")]
for k, m in med.items():
    print(k)
    for c in sorted(m):
        print(f"    {c:28s} {m[c]:.6g}")
    for name, a, b in ratios:
        if a in m and b in m and m[b]:
            print(f"  = {name:36s} {m[a] / m[b]:.3f}")

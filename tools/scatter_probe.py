"""bin_scatter phase proportions from the timing probe build (profiles/r06_v9_scatter_phase_probe.txt):

    EXTRA=-DMFN_SCATTER_PROBE bash tools/build_variant.sh - probe
    MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/probe.so python tools/scatter_probe.py mf128 out.txt

runs bench.py's step (50 steps) in-process, then reads the kernel's phase counters
(mfnerf_scatter_probe_read, exported by the probe build only) and writes the proportions to out.txt.
"""
import ctypes, json, sys, io, contextlib
sys.path.insert(0, ".")
import bench
preset = sys.argv[1]
rc = bench.main(["--steps", "50", "--warmup", "5", "--no-cpu-baseline", "--preset", preset])
res = open(sys.argv[2], "w")
lib = sys.modules["mfnerf._lib"].load()
buf = (ctypes.c_ulonglong * 32)()
assert lib.mfnerf_scatter_probe_read(buf) == 0
g = list(buf)
n = g[15]
names = ["place", "stage+count next", "barrier 1", "store", "scan", "barrier 2"]
for o, w in ((0, "wave 0"), (6, "wave 8")):
    tot = sum(g[o:o + 6])
    print(file=res, end=f"{preset} {w}: cycles per unit launch {tot / n:.0f}; " +
          ", ".join(f"{names[k]} {100 * g[o + k] / tot:.1f}%" for k in range(6)) + "\n")
print(preset, "unit launches", n, file=res)
cl = g[16:32]
tc = sum(cl)
print(preset, "wave 8 count cycles per unit launch by level index j:", ", ".join(f"j{j} {cl[j] / n:.0f}" for j in range(16) if cl[j]), f"(sum {tc / n:.0f})", file=res)
if hasattr(lib, "mfnerf_accum_probe_read"):
    ab = (ctypes.c_ulonglong * 8)()
    assert lib.mfnerf_accum_probe_read(ab) == 0
    a = list(ab)
    na = max(1, a[7])
    tot = sum(a[:6])
    names = ["setup", "copies issued", "copy wait", "adds", "last barrier", "adam"]
    print(f"{preset} bin_accum wave 0: cycles per partition workgroup {tot / na:.0f} ({na} workgroups); " +
          ", ".join(f"{names[k]} {100 * a[k] / tot:.1f}%" for k in range(6)), file=res)

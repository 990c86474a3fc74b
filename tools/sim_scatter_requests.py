"""CPU model of grid_bw's memory-side atomic request count (one request per distinct 64-B line of a
wave-instruction; lanes on one line are free) on the bench workload: the oracle march of an
8192-ray batch of the ball scene, Lego hash layout.  Prints requests per sample per level for the
current kernel's lane layout and for alternative orderings / aggregation windows.

    python tools/sim_scatter_requests.py [--rays 8192]
"""
import argparse
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]

P1, P2 = np.uint64(2654435761), np.uint64(805459861)


def march(n_rays, seed=0):
    from mfnerf import synthetic
    from oracle import vren_oracle as O
    poses = synthetic.camera_poses()
    o, d = synthetic.random_rays(n_rays, poses, seed=seed)
    bf = synthetic.packbits_np(synthetic.ball_density_grid(), 0.01 * 1024 / math.sqrt(3))
    _, ht, _ = O.ray_aabb_intersect(o, d, torch.zeros(1, 3), torch.full((1, 3), 0.5), 1)
    ht[(ht[:, 0, 0] >= 0) & (ht[:, 0, 0] < 0.01), 0, 0] = 0.01
    g = torch.Generator().manual_seed(seed)
    ra, x, dd, de, ts, cnt = O.raymarching_train(o, d, ht[:, 0].contiguous(), bf, 1, 0.5, 0.0,
                                                 torch.rand(n_rays, generator=g), 128, 1024)
    n = int(cnt[0])
    return x[:n].numpy().astype(np.float32), ra.numpy()


def corners(xn, layout, l):
    """(n, 8) table entry index of the 8 corners of level l (corner c: x+(c&1), y+(c>>1&1), z+(c>>2&1))."""
    s = np.float32(layout.scales[l])
    pos = (s * xn.astype(np.float32) + np.float32(0.5)).astype(np.float32)  # fmaf ~ fp32 here (model)
    g = np.floor(pos).astype(np.int64)
    res, size = layout.res[l], layout.sizes[l]
    out = np.empty((len(xn), 8), np.int64)
    for c in range(8):
        gx, gy, gz = g[:, 0] + (c & 1), g[:, 1] + ((c >> 1) & 1), g[:, 2] + ((c >> 2) & 1)
        if res ** 3 <= size:
            idx = gx + gy * res + gz * res * res
        else:
            ux, uy, uz = (gx.astype(np.uint64), gy.astype(np.uint64), gz.astype(np.uint64))
            idx = ((ux ^ (uy * P1) ^ (uz * P2)) & np.uint64(0xFFFFFFFF)).astype(np.int64)
        out[:, c] = idx % size
    return out


def current_requests(idx, chunk=16):
    """The kernel's layout: 16 consecutive samples per wave; per (level, yz) one instruction whose
    lanes are (s, xb, f); run heads of equal idx per xb stream issue; count distinct lines."""
    n = idx.shape[0]
    pad = (-n) % chunk
    req = 0
    for yz in range(4):
        c0, c1 = idx[:, 2 * yz], idx[:, 2 * yz + 1]
        for cc in (c0, c1):
            pass
        a = np.concatenate([c0, np.full(pad, -1)]).reshape(-1, chunk)
        b = np.concatenate([c1, np.full(pad, -1)]).reshape(-1, chunk)
        heads_a = np.ones_like(a, bool); heads_a[:, 1:] = a[:, 1:] != a[:, :-1]
        heads_b = np.ones_like(b, bool); heads_b[:, 1:] = b[:, 1:] != b[:, :-1]
        la = np.where(heads_a & (a >= 0), a // 8, -1)  # 8 entries (F=2 fp32) per 64-B line
        lb = np.where(heads_b & (b >= 0), b // 8, -1)
        lines = np.concatenate([la, lb], 1)
        lines.sort(1)
        distinct = (lines[:, 1:] != lines[:, :-1]) & (lines[:, 1:] >= 0)
        req += int(distinct.sum() + (lines[:, 0] >= 0).sum())
    return req


def window_distinct_lines(idx, window):
    """Perfect aggregation inside windows of `window` consecutive samples: one request per distinct
    line per window."""
    n = idx.shape[0]
    w = np.arange(n) // window
    key = w[:, None] * (1 << 24) + idx // 8
    return len(np.unique(key.ravel()))


def morton_key(xn, bits=10):
    q = np.clip((xn * (1 << bits)).astype(np.int64), 0, (1 << bits) - 1)
    k = np.zeros(len(xn), np.int64)
    for b in range(bits):
        for a in range(3):
            k |= ((q[:, a] >> b) & 1) << (3 * b + a)
    return k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=8192)
    args = ap.parse_args()
    from mfnerf.grid import GridLayout
    b = math.exp(math.log(2048 * 0.5 / 16) / 15)
    lay = GridLayout(16, 2, 19, 16, b)
    x, ra = march(args.rays)
    xn = ((x + np.float32(0.5)) / np.float32(1.0)).astype(np.float32)
    n = len(xn)
    print(f"{n} samples, {n / args.rays:.1f} per ray")
    perm = np.argsort(morton_key(xn, 10), kind="stable")
    tot = {}
    print("lvl  res   cur/s  win64/s win256/s  sorted:cur/s  sortwin256/s  global/s")
    for l in range(16):
        idx = corners(xn, lay, l)
        r = {
            "cur": current_requests(idx),
            "w64": window_distinct_lines(idx, 64),
            "w256": window_distinct_lines(idx, 256),
            "scur": current_requests(idx[perm]),
            "sw256": window_distinct_lines(idx[perm], 256),
            "glob": window_distinct_lines(idx, n),
        }
        for k, v in r.items():
            tot[k] = tot.get(k, 0) + v
        print(f"{l:3d} {lay.res[l]:5d} " + "  ".join(f"{r[k] / n:7.2f}" for k in ("cur", "w64", "w256", "scur", "sw256", "glob")))
    print("sum          " + "  ".join(f"{tot[k] / n:7.2f}" for k in ("cur", "w64", "w256", "scur", "sw256", "glob")))


if __name__ == "__main__":
    main()

"""Seeded synthetic inputs of the hot path, on any device.

* rays: 100 cameras on a sphere of radius 1.5 looking at the origin, Lego intrinsics
  (fx = fy = 1111.111, cx = cy = 400, 800x800), one random pixel per ray, directions
  unnormalised in camera space (z = 1) exactly like datasets/ray_utils.py:8-70 builds them.
* occupancy: a seeded union of solid balls inside [-0.5, 0.5]^3 written into the (C, G^3)
  density grid at each cell's Morton index and packed with the reference's threshold;
  the defaults give ~63 ray-march samples per ray at the Lego batch (SURVEY.md 8d asks 60-68).
There is no dataset download in this environment; these stand in for Lego.
"""
import math

import numpy as np
import torch

LEGO_W = LEGO_H = 800
LEGO_F = 0.5 * 800 / math.tan(0.5 * 0.6911112)  # 1111.111


def camera_poses(n_cams=100, radius=1.5, seed=0):
    """(n_cams, 3, 4) c2w in the [right down front] camera convention (ray_utils.py:24-35)."""
    g = np.random.default_rng(seed)
    poses = []
    for _ in range(n_cams):
        v = g.normal(size=3)
        v /= np.linalg.norm(v)
        o = v * radius
        fwd = -o / np.linalg.norm(o)                 # camera +z looks at the origin
        tmp = np.array([0.0, 0.0, 1.0]) if abs(fwd[2]) < 0.9 else np.array([1.0, 0.0, 0.0])
        right = np.cross(tmp, fwd); right /= np.linalg.norm(right)
        down = np.cross(fwd, right)
        poses.append(np.stack([right, down, fwd, o], 1))
    return torch.tensor(np.stack(poses), dtype=torch.float32)


def random_rays(n_rays, poses, seed=0, device="cpu", W=LEGO_W, H=LEGO_H, focal=LEGO_F):
    """One random pixel of a random camera per ray -> rays_o, rays_d (N,3) f32 (get_rays semantics)."""
    g = torch.Generator().manual_seed(seed)
    cam = torch.randint(len(poses), (n_rays,), generator=g)
    pix = torch.randint(W * H, (n_rays,), generator=g)
    u = (pix % W).float()
    v = (pix // W).float()
    dirs_c = torch.stack([(u - W / 2 + 0.5) / focal, (v - H / 2 + 0.5) / focal, torch.ones_like(u)], -1)
    c2w = poses[cam]
    rays_d = (dirs_c[:, None, :] @ c2w[:, :, :3].transpose(1, 2))[:, 0]
    rays_o = c2w[:, :, 3].contiguous()
    return rays_o.to(device), rays_d.contiguous().to(device)


def _morton3(x, y, z):
    def expand(v):
        v = (v * 0x00010001) & 0xFF0000FF
        v = (v * 0x00000101) & 0x0F00F00F
        v = (v * 0x00000011) & 0xC30C30C3
        v = (v * 0x00000005) & 0x49249249
        return v
    return expand(x) | (expand(y) << 1) | (expand(z) << 2)


def ball_density_grid(G=128, cascades=1, scale=0.5, n_balls=12, radius=(0.065, 0.18), seed=0, occupied=10.0):
    """(C, G^3) f32 density grid (index = mip*G^3 + morton), `occupied` inside a union of balls."""
    g = np.random.default_rng(seed)
    centers = g.uniform(-0.5 + radius[1], 0.5 - radius[1], size=(n_balls, 3))
    radii = g.uniform(radius[0], radius[1], size=n_balls)
    return balls_to_grid(centers, radii, G=G, cascades=cascades, scale=scale, occupied=occupied)


def balls_to_grid(centers, radii, G=128, cascades=1, scale=0.5, occupied=10.0):
    """(C, G^3) f32 density grid, `occupied` in the cells whose centre lies inside a ball."""
    centers, radii = np.asarray(centers, np.float64), np.asarray(radii, np.float64)
    grid = np.zeros((cascades, G ** 3), np.float32)
    ii = np.arange(G, dtype=np.int64)
    x, y, z = np.meshgrid(ii, ii, ii, indexing="ij")
    x, y, z = x.ravel(), y.ravel(), z.ravel()
    idx = _morton3(x, y, z)
    for c in range(cascades):
        s = min(2 ** (c - 1), scale)
        pw = np.stack([(x + 0.5) / G * 2 - 1, (y + 0.5) / G * 2 - 1, (z + 0.5) / G * 2 - 1], 1) * s
        inside = np.zeros(len(x), bool)
        for cc, rr in zip(centers, radii):
            inside |= ((pw - cc) ** 2).sum(1) <= rr * rr
        grid[c, idx[inside]] = occupied
    return torch.from_numpy(grid)


def packbits_np(grid, thr):
    """Reference packbits (raymarching.cu:122-141): bit i of byte n = grid[8n+i] > thr."""
    bits = (grid.reshape(-1).numpy() > thr)
    return torch.from_numpy(np.packbits(bits, bitorder="little"))

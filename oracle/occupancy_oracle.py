"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's occupancy-grid refresh, used by
tests/ as the checker for mfnerf_occupancy_* (never imported by the product path).

Follows models/networks.py (lly00412/MF-NeRF):
  get_all_cells                     :157-166  (warm-up: every cell, morton index of grid_coords)
  sample_uniform_and_occupied_cells :168-192  (M uniform + M drawn from nonzero(grid > thr))
  update_density_grid               :242-271  (jittered cell points, tmp scatter, decay/max, mean, packbits)
The random draws (torch.randint / torch.rand) cannot be reproduced bit for bit by the device's
counter-based generator, so the draw step is checked through properties (cell_points_ok); the
deterministic part (update) is restated exactly.  Parity pinned by the reference's own Python
only through these semantics (no reference test covers this path).
"""
import numpy as np
import torch

from . import vren_oracle


def cell_centers(cell_idx, cascades, G, scale):
    """(coords/(G-1)*2-1)*(s-half) for flat indices cascade*G^3 + morton (networks.py:251-254)."""
    cell_idx = torch.as_tensor(cell_idx).long()
    c = cell_idx // G ** 3
    m = (cell_idx % G ** 3).int().contiguous()
    coords = vren_oracle.morton3D_invert(m).float()
    s = torch.minimum(torch.exp2(c.float() - 1), torch.tensor(float(scale)))
    half = s / G
    return (coords / (G - 1) * 2 - 1) * (s - half)[:, None], half


def cell_points_ok(xyz, cell_idx, cascades, G, scale, atol=1e-6):
    """Every point lies within half a cell of its cell's centre (the jitter, networks.py:255)."""
    ctr, half = cell_centers(cell_idx, cascades, G, scale)
    return bool(((xyz - ctr).abs() <= half[:, None] + atol).all())


def update(density_grid, sigmas, cell_idx, decay=0.95, count_grid=None, density_threshold=0.01 * 1024 / 3 ** 0.5):
    """networks.py:259-271 given the probed (cell, sigma) pairs; cell_idx < 0 are skipped.
    Returns (new_grid (C,G^3) f32, thr f32, bitfield u8).  Duplicate cells: the last pair wins
    here; the device keeps one of them (the reference's index_put is equally unordered)."""
    g = density_grid.clone()
    tmp = torch.zeros_like(g).reshape(-1)
    keep = cell_idx >= 0
    tmp[cell_idx[keep].long()] = sigmas[keep]
    tmp = tmp.reshape(g.shape)
    if count_grid is not None:
        decay = torch.clamp(decay ** (1 / count_grid), 0.1, 0.95)
    g = torch.where(g < 0, g, torch.maximum(g * decay, tmp))
    pos = g[g > 0]
    mean = pos.double().mean().float().item() if pos.numel() else float("nan")
    thr = min(mean, density_threshold)
    bf = torch.zeros(g.numel() // 8, dtype=torch.uint8)
    vren_oracle.packbits(g.contiguous(), thr, bf)
    return g, thr, bf

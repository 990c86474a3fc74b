"""NGP field model of models/networks.py:12-271 on the gfx950 kernels.

Same constructor (scale, hparams, rgb_act), buffers (center, xyz_min, xyz_max, half_size,
density_bitfield; plus density_grid and grid_coords, which the reference's train.py:78-81
registers on the model), parameters (xyz_encoder.params, rgb_net.params in tcnn layout) and
methods (density, forward, get_all_cells, sample_uniform_and_occupied_cells,
mark_invisible_cells, update_density_grid).  forward/density run the fused field kernels
(grid encode -> MFMA MLPs -> TruncExp/SH4/sigmoid) instead of three tcnn modules.
The HDR path (rgb_act='None', tonemappers) is out of scope.
"""
import numpy as np
import torch
from einops import rearrange
from torch import nn

from . import tcnn, vren
from .field import NGPDensityFunction, NGPFieldFunction
from .rendering import NEAR_DISTANCE


def _meshgrid3d(G, device=None):
    """kornia create_meshgrid3d(G, G, G, False, dtype=int32).reshape(-1, 3) ordering (train.py:80-81)."""
    r = torch.arange(G, dtype=torch.int32, device=device)
    d, h, w = torch.meshgrid(r, r, r, indexing="ij")
    return torch.stack([d, h, w], -1).reshape(-1, 3)


@torch.no_grad()
def mark_invisible_cells(density_grid, grid_coords, scale, K, poses, img_wh, chunk=64 ** 3):
    """networks.py:199-240 on a (C, G^3) density grid (in place): cells seen by no camera, or too
    near one, get -1 (never updated again), the others 0.  Returns count_grid (the fraction of
    cameras seeing each cell; used by the erode option of the occupancy refresh)."""
    cascades, G = density_grid.shape[0], round(density_grid.shape[1] ** (1 / 3))
    count_grid = torch.zeros_like(density_grid)
    N_cams = poses.shape[0]
    w2c_R = rearrange(poses[:, :3, :3], "n a b -> n b a")
    w2c_T = -w2c_R @ poses[:, :3, 3:]
    indices = vren.morton3D(grid_coords).long()
    for c in range(cascades):
        for i in range(0, len(indices), chunk):
            xyzs = grid_coords[i:i + chunk] / (G - 1) * 2 - 1
            s = min(2 ** (c - 1), scale)
            half_grid_size = s / G
            xyzs_w = (xyzs * (s - half_grid_size)).T
            xyzs_c = w2c_R @ xyzs_w + w2c_T
            uvd = K @ xyzs_c
            uv = uvd[:, :2] / uvd[:, 2:]
            in_image = (uvd[:, 2] >= 0) & (uv[:, 0] >= 0) & (uv[:, 0] < img_wh[0]) & \
                       (uv[:, 1] >= 0) & (uv[:, 1] < img_wh[1])
            covered_by_cam = (uvd[:, 2] >= NEAR_DISTANCE) & in_image
            count_grid[c, indices[i:i + chunk]] = count = covered_by_cam.sum(0) / N_cams
            too_near_to_cam = (uvd[:, 2] < NEAR_DISTANCE) & in_image
            too_near_to_any_cam = too_near_to_cam.any(0)
            valid_mask = (count > 0) & (~too_near_to_any_cam)
            density_grid[c, indices[i:i + chunk]] = torch.where(valid_mask, 0., -1.)
    return count_grid


class NGP(nn.Module):
    def __init__(self, scale, hparams, rgb_act="Sigmoid"):
        super().__init__()
        if rgb_act != "Sigmoid":
            raise NotImplementedError("the HDR/exposure path (rgb_act='None') is out of scope")
        self.rgb_act = rgb_act
        self.scale = scale
        self.register_buffer("center", torch.zeros(1, 3))
        self.register_buffer("xyz_min", -torch.ones(1, 3) * scale)
        self.register_buffer("xyz_max", torch.ones(1, 3) * scale)
        self.register_buffer("half_size", (self.xyz_max - self.xyz_min) / 2)

        self.cascades = max(1 + int(np.ceil(np.log2(2 * scale))), 1)
        self.grid_size = 128
        self.register_buffer("density_bitfield",
                             torch.zeros(self.cascades * self.grid_size ** 3 // 8, dtype=torch.uint8))
        G = self.grid_size
        self.register_buffer("density_grid", torch.zeros(self.cascades, G ** 3))
        self.register_buffer("grid_coords", _meshgrid3d(G))

        L, F, log2_T, N_min = hparams.L, hparams.F, hparams.T, hparams.N_min
        N_tables = getattr(hparams, "N_tables", 1)
        b = np.exp(np.log(hparams.N_max * scale / N_min) / (L - 1))
        self.rgb_width = hparams.rgb_channels
        if L * F != 32:
            raise NotImplementedError("the fused field head takes L*F = 32 grid features (the reference's L=16, F=2)")
        if hparams.rgb_layers != 2:
            raise NotImplementedError("the fused field head implements rgb_layers=2 (the reference default)")
        self.xyz_encoder = tcnn.NetworkWithInputEncoding(
            n_input_dims=3, n_output_dims=16,
            encoding_config={"otype": f"{hparams.grid}Grid", "type": hparams.grid, "n_levels": L,
                             "n_features_per_level": F, "log2_hashmap_size": log2_T, "base_resolution": N_min,
                             "n_tables": N_tables, "per_level_scale": b, "interpolation": "Linear"},
            network_config={"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None",
                            "n_neurons": 64, "n_hidden_layers": 1})
        self.dir_encoder = tcnn.Encoding(n_input_dims=3,
                                         encoding_config={"otype": "SphericalHarmonics", "degree": 4})
        self.rgb_net = tcnn.Network(
            n_input_dims=32, n_output_dims=3,
            network_config={"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": self.rgb_act,
                            "n_neurons": hparams.rgb_channels, "n_hidden_layers": hparams.rgb_layers})
        self.layout, self.desc = self.xyz_encoder.layout, self.xyz_encoder.desc
        s = np.float32(scale)
        self._x_min = float(-s)
        self._x_range = float(np.float32(s) - np.float32(-s))

    def density(self, x, return_feat=False):
        """networks.py:96-109 (return_feat is served by forward(); the feature is fused away)."""
        if return_feat:
            raise NotImplementedError("return_feat: the fused head does not materialise h; use forward()")
        return NGPDensityFunction.apply(x, self.xyz_encoder.params, self.rgb_net.params, self.layout, self.desc,
                                        self._x_min, self._x_range, self.rgb_width)

    def forward(self, x, d, **kwargs):
        """networks.py:134-155 -> sigmas (N) f32, rgbs (N,3)."""
        return NGPFieldFunction.apply(x, d, self.xyz_encoder.params, self.rgb_net.params, self.layout, self.desc,
                                      self._x_min, self._x_range, self.rgb_width)

    @torch.no_grad()
    def get_all_cells(self):
        indices = vren.morton3D(self.grid_coords).long()
        return [(indices, self.grid_coords)] * self.cascades

    @torch.no_grad()
    def sample_uniform_and_occupied_cells(self, M, density_threshold):
        cells = []
        for c in range(self.cascades):
            coords1 = torch.randint(self.grid_size, (M, 3), dtype=torch.int32, device=self.density_grid.device)
            indices1 = vren.morton3D(coords1).long()
            indices2 = torch.nonzero(self.density_grid[c] > density_threshold)[:, 0]
            if len(indices2) > 0:
                rand_idx = torch.randint(len(indices2), (M,), device=self.density_grid.device)
                indices2 = indices2[rand_idx]
            coords2 = vren.morton3D_invert(indices2.int().contiguous())
            cells += [(torch.cat([indices1, indices2]), torch.cat([coords1, coords2]))]
        return cells

    @torch.no_grad()
    def mark_invisible_cells(self, K, poses, img_wh, chunk=64 ** 3):
        """networks.py:199-240."""
        self.count_grid = mark_invisible_cells(self.density_grid, self.grid_coords, self.scale, K, poses, img_wh,
                                               chunk)

    @torch.no_grad()
    def update_density_grid(self, density_threshold, warmup=False, decay=0.95, erode=False):
        """networks.py:242-271."""
        density_grid_tmp = torch.zeros_like(self.density_grid)
        if warmup:
            cells = self.get_all_cells()
        else:
            cells = self.sample_uniform_and_occupied_cells(self.grid_size ** 3 // 4, density_threshold)
        for c in range(self.cascades):
            indices, coords = cells[c]
            s = min(2 ** (c - 1), self.scale)
            half_grid_size = s / self.grid_size
            xyzs_w = (coords / (self.grid_size - 1) * 2 - 1) * (s - half_grid_size)
            xyzs_w += (torch.rand_like(xyzs_w) * 2 - 1) * half_grid_size
            density_grid_tmp[c, indices] = self.density(xyzs_w)
        if erode:
            decay = torch.clamp(decay ** (1 / self.count_grid), 0.1, 0.95)
        self.density_grid = torch.where(self.density_grid < 0, self.density_grid,
                                        torch.maximum(self.density_grid * decay, density_grid_tmp))
        mean_density = self.density_grid[self.density_grid > 0].mean().item()
        vren.packbits(self.density_grid, min(mean_density, density_threshold), self.density_bitfield)

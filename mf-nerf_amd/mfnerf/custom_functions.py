"""autograd.Function surface of models/custom_functions.py, over the gfx950 `vren` ops.

Same class names, apply() signatures and outputs as the reference (custom_functions.py:8-173).
Inputs are cast to fp32 like the reference's custom_fwd(cast_inputs=torch.float32).
RaySphereIntersector (no caller in the reference) is out of scope.
"""
import torch

from . import vren


def _f32(*ts):
    return [t.float() if isinstance(t, torch.Tensor) and t.is_floating_point() else t for t in ts]


class RayAABBIntersector(torch.autograd.Function):
    """custom_functions.py:8-29: (rays_o, rays_d, centers, half_sizes, max_hits) ->
    hits_cnt (N) i32, hits_t (N,max_hits,2) near->far (-1 no hit), hits_voxel_idx (N,max_hits) i64."""

    @staticmethod
    def forward(ctx, rays_o, rays_d, center, half_size, max_hits):
        rays_o, rays_d, center, half_size = _f32(rays_o, rays_d, center, half_size)
        return tuple(vren.ray_aabb_intersect(rays_o.contiguous(), rays_d.contiguous(), center.contiguous(),
                                             half_size.contiguous(), max_hits))


class RayMarcher(torch.autograd.Function):
    """custom_functions.py:55-112: march rays through the occupancy bitfield.

    Outputs rays_a (N_rays,3) = (ray_idx, start_idx, N_samples), xyzs (N,3), dirs (N,3), deltas (N),
    ts (N), total_samples (0-d).  rays_a rows are in ray order (the reference's are in atomicAdd
    order; every consumer indexes through rays_a).  Like the reference this reads counter[0] on the
    host (one sync); the fused engine (mfnerf.engine) keeps it on the device instead."""

    @staticmethod
    def forward(ctx, rays_o, rays_d, hits_t, density_bitfield, cascades, scale, exp_step_factor, grid_size,
                max_samples):
        rays_o, rays_d, hits_t = _f32(rays_o, rays_d, hits_t)
        noise = torch.rand_like(rays_o[:, 0])
        rays_a, xyzs, dirs, deltas, ts, counter = vren.raymarching_train(
            rays_o, rays_d, hits_t, density_bitfield, cascades, scale, exp_step_factor, noise, grid_size,
            max_samples)
        total_samples = counter[0]
        n = int(total_samples)
        xyzs, dirs, deltas, ts = xyzs[:n], dirs[:n], deltas[:n], ts[:n]
        ctx.save_for_backward(rays_a, ts)
        return rays_a, xyzs, dirs, deltas, ts, total_samples

    @staticmethod
    def backward(ctx, dL_drays_a, dL_dxyzs, dL_ddirs, dL_ddeltas, dL_dts, dL_dtotal_samples):
        # segment_csr restated as index_add over the CSR segments (custom_functions.py:103-112)
        rays_a, ts = ctx.saved_tensors
        N = rays_a.shape[0]
        seg = torch.repeat_interleave(torch.arange(N, device=ts.device), rays_a[:, 2])
        ray_of = rays_a[:, 0][seg]
        dL_drays_o = torch.zeros(N, 3, device=ts.device, dtype=dL_dxyzs.dtype)
        dL_drays_o.index_add_(0, ray_of, dL_dxyzs)
        dL_drays_d = torch.zeros(N, 3, device=ts.device, dtype=dL_dxyzs.dtype)
        dL_drays_d.index_add_(0, ray_of, dL_dxyzs * ts[:, None] + dL_ddirs)
        return dL_drays_o, dL_drays_d, None, None, None, None, None, None, None


class VolumeRenderer(torch.autograd.Function):
    """custom_functions.py:115-159: front-to-back compositing with early termination.
    Outputs total_samples.sum() (effective samples), opacity, depth, rgb (N_rays,3), ws (N)."""

    @staticmethod
    def forward(ctx, sigmas, rgbs, deltas, ts, rays_a, T_threshold):
        sigmas, rgbs, deltas, ts = [t.float().contiguous() for t in (sigmas, rgbs, deltas, ts)]
        total_samples, opacity, depth, rgb, ws = vren.composite_train_fw(sigmas, rgbs, deltas, ts, rays_a,
                                                                         T_threshold)
        ctx.save_for_backward(sigmas, rgbs, deltas, ts, rays_a, opacity, depth, rgb, ws)
        ctx.T_threshold = T_threshold
        return total_samples.sum(), opacity, depth, rgb, ws

    @staticmethod
    def backward(ctx, dL_dtotal_samples, dL_dopacity, dL_ddepth, dL_drgb, dL_dws):
        sigmas, rgbs, deltas, ts, rays_a, opacity, depth, rgb, ws = ctx.saved_tensors
        z = lambda t, like: torch.zeros_like(like) if t is None else t.float().contiguous()  # noqa: E731
        dL_dsigmas, dL_drgbs = vren.composite_train_bw(z(dL_dopacity, opacity), z(dL_ddepth, depth),
                                                       z(dL_drgb, rgb), z(dL_dws, ws), sigmas, rgbs, ws, deltas,
                                                       ts, rays_a, opacity, depth, rgb, ctx.T_threshold)
        return dL_dsigmas, dL_drgbs, None, None, None, None


class TruncExp(torch.autograd.Function):
    """custom_functions.py:162-173: exp forward, exp(clamp(x,-15,15)) backward."""

    @staticmethod
    def forward(ctx, x):
        x = x.float()
        ctx.save_for_backward(x)
        return torch.exp(x)

    @staticmethod
    def backward(ctx, dL_dout):
        x = ctx.saved_tensors[0]
        return dL_dout * torch.exp(x.clamp(-15, 15))

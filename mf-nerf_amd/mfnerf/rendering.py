"""models/rendering.py restated over the gfx950 ops: render() and its train/test paths.

Same entry point, constants, kwargs and result keys as the reference (rendering.py:1-163):
near clamp of the AABB hit (:29), the progressive test-time march (:46-118, including
N_samples = max(min(N//N_alive, 64), min_samples)) and the background blend (:112-116,
:153-161).
"""
import torch
from einops import rearrange

from . import vren
from .custom_functions import RayAABBIntersector, RayMarcher, VolumeRenderer

MAX_SAMPLES = 1024
NEAR_DISTANCE = 0.01


def render(model, rays_o, rays_d, **kwargs):
    """rendering.py:11-43 (the reference runs it under torch.cuda.amp.autocast())."""
    with torch.autocast("cuda", enabled=rays_o.is_cuda):
        return _render(model, rays_o, rays_d, **kwargs)


def _render(model, rays_o, rays_d, **kwargs):
    rays_o = rays_o.contiguous()
    rays_d = rays_d.contiguous()
    _, hits_t, _ = RayAABBIntersector.apply(rays_o, rays_d, model.center, model.half_size, 1)
    hits_t[(hits_t[:, 0, 0] >= 0) & (hits_t[:, 0, 0] < NEAR_DISTANCE), 0, 0] = NEAR_DISTANCE

    render_func = _render_rays_test if kwargs.get("test_time", False) else _render_rays_train
    results = render_func(model, rays_o, rays_d, hits_t, **kwargs)
    for k, v in results.items():
        if kwargs.get("to_cpu", False):
            v = v.cpu()
            if kwargs.get("to_numpy", False):
                v = v.numpy()
        results[k] = v
    return results


@torch.no_grad()
def _render_rays_test(model, rays_o, rays_d, hits_t, **kwargs):
    """rendering.py:46-118: march alive rays N_samples at a time until they converge."""
    exp_step_factor = kwargs.get("exp_step_factor", 0.0)
    results = {}
    N_rays = len(rays_o)
    device = rays_o.device
    opacity = torch.zeros(N_rays, device=device)
    depth = torch.zeros(N_rays, device=device)
    rgb = torch.zeros(N_rays, 3, device=device)

    samples = total_samples = 0
    alive_indices = torch.arange(N_rays, device=device)
    min_samples = 1 if exp_step_factor == 0 else 4

    while samples < kwargs.get("max_samples", MAX_SAMPLES):
        N_alive = len(alive_indices)
        if N_alive == 0:
            break
        N_samples = max(min(N_rays // N_alive, 64), min_samples)
        samples += N_samples

        xyzs, dirs, deltas, ts, N_eff_samples = vren.raymarching_test(
            rays_o, rays_d, hits_t[:, 0], alive_indices, model.density_bitfield, model.cascades, model.scale,
            exp_step_factor, model.grid_size, MAX_SAMPLES, N_samples)
        total_samples += N_eff_samples.sum()
        xyzs = rearrange(xyzs, "n1 n2 c -> (n1 n2) c")
        dirs = rearrange(dirs, "n1 n2 c -> (n1 n2) c")
        valid_mask = ~torch.all(dirs == 0, dim=1)
        # the valid samples' indices once (one host sync), instead of a mask sum plus a nonzero per
        # boolean index below; same values as the reference's masked assignments
        valid = valid_mask.nonzero()[:, 0]
        if len(valid) == 0:
            break

        sigmas = torch.zeros(len(xyzs), device=device)
        rgbs = torch.zeros(len(xyzs), 3, device=device)
        _sigmas, _rgbs = model(xyzs.index_select(0, valid), dirs.index_select(0, valid), **kwargs)
        sigmas.index_copy_(0, valid, _sigmas.float())
        rgbs.index_copy_(0, valid, _rgbs.float())
        sigmas = rearrange(sigmas, "(n1 n2) -> n1 n2", n2=N_samples)
        rgbs = rearrange(rgbs, "(n1 n2) c -> n1 n2 c", n2=N_samples)

        vren.composite_test_fw(sigmas.contiguous(), rgbs.contiguous(), deltas, ts, hits_t[:, 0], alive_indices,
                               kwargs.get("T_threshold", 1e-4), N_eff_samples, opacity, depth, rgb)
        alive_indices = alive_indices[alive_indices >= 0]

    results["opacity"] = opacity
    results["depth"] = depth
    results["rgb"] = rgb
    results["total_samples"] = total_samples

    rgb_bg = torch.ones(3, device=device) if exp_step_factor == 0 else torch.zeros(3, device=device)
    results["rgb"] += rgb_bg * rearrange(1 - opacity, "n -> n 1")
    return results


def _render_rays_train(model, rays_o, rays_d, hits_t, **kwargs):
    """rendering.py:121-163."""
    exp_step_factor = kwargs.get("exp_step_factor", 0.0)
    results = {}

    (rays_a, xyzs, dirs, results["deltas"], results["ts"], results["rm_samples"]) = RayMarcher.apply(
        rays_o, rays_d, hits_t[:, 0], model.density_bitfield, model.cascades, model.scale, exp_step_factor,
        model.grid_size, MAX_SAMPLES)

    for k, v in kwargs.items():
        if isinstance(v, torch.Tensor):
            kwargs[k] = torch.repeat_interleave(v[rays_a[:, 0]], rays_a[:, 2], 0)
    sigmas, rgbs = model(xyzs, dirs, **kwargs)

    (results["vr_samples"], results["opacity"], results["depth"], results["rgb"], results["ws"]) = \
        VolumeRenderer.apply(sigmas, rgbs.contiguous(), results["deltas"], results["ts"], rays_a,
                             kwargs.get("T_threshold", 1e-4))
    results["rays_a"] = rays_a

    if exp_step_factor == 0:
        rgb_bg = torch.ones(3, device=rays_o.device)
    elif kwargs.get("random_bg", False):
        rgb_bg = torch.rand(3, device=rays_o.device)
    else:
        rgb_bg = torch.zeros(3, device=rays_o.device)
    results["rgb"] = results["rgb"] + rgb_bg * rearrange(1 - results["opacity"], "n -> n 1")
    return results

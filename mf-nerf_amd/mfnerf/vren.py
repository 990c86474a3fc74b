"""`vren`-compatible op module backed by libmfnerf_hip.so (gfx950 HIP kernels).

Same function names, argument order, return layout and error behaviour as the reference's
pybind module (models/csrc/binding.cpp:234-250): CUDA + contiguous inputs are required
(RuntimeError otherwise, as CHECK_INPUT raises c10::Error), outputs are fresh tensors on the
input's device, and the in-place mutators (packbits, raymarching_test's hits_t[:,0],
composite_test_fw's alive/opacity/depth/rgb) mutate their arguments.

A maintainer swaps it in with `sys.modules['vren'] = mfnerf.vren`.
ray_sphere_intersect has no caller in the reference and is out of scope.
"""
import torch

from ._lib import call, check_input, ptr, stream

_f32, _i32, _i64, _u8 = torch.float32, torch.int32, torch.int64, torch.uint8


def ray_aabb_intersect(rays_o, rays_d, centers, half_sizes, max_hits):
    """intersection.cu:59-100 -> [hit_cnt (N) i32, hits_t (N,max_hits,2), hits_voxel_idx (N,max_hits) i64]."""
    for n, t in (("rays_o", rays_o), ("rays_d", rays_d), ("centers", centers), ("half_sizes", half_sizes)):
        check_input(n, t, _f32)
    N, V = rays_o.shape[0], centers.shape[0]
    dev = rays_o.device
    hit_cnt = torch.empty(N, dtype=_i32, device=dev)
    hits_t = torch.empty(N, max_hits, 2, dtype=_f32, device=dev)
    idx = torch.empty(N, max_hits, dtype=_i64, device=dev)
    call("mfnerf_ray_aabb_intersect", ptr(rays_o), ptr(rays_d), ptr(centers), ptr(half_sizes), N, V, int(max_hits),
         ptr(hit_cnt), ptr(hits_t), ptr(idx), stream())
    return [hit_cnt, hits_t, idx]


def ray_sphere_intersect(rays_o, rays_d, centers, radii, max_hits):
    raise NotImplementedError("ray_sphere_intersect has no caller in MF-NeRF and is out of scope (SURVEY.md 2.2)")


def morton3D(coords):
    check_input("coords", coords, _i32)
    out = torch.empty(coords.shape[0], dtype=_i32, device=coords.device)
    call("mfnerf_morton3d", ptr(coords), coords.shape[0], ptr(out), stream())
    return out


def morton3D_invert(indices):
    check_input("indices", indices, _i32)
    out = torch.empty(indices.shape[0], 3, dtype=_i32, device=indices.device)
    call("mfnerf_morton3d_invert", ptr(indices), indices.shape[0], ptr(out), stream())
    return out


def packbits(density_grid, density_threshold, density_bitfield):
    """In place on density_bitfield; density_threshold may be a python float or a 0-d CUDA tensor."""
    check_input("density_grid", density_grid, _f32)
    check_input("density_bitfield", density_bitfield, _u8)
    if density_grid.numel() < 8 * density_bitfield.numel():
        raise RuntimeError("density_grid too small for density_bitfield")
    thr_dev = None
    if isinstance(density_threshold, torch.Tensor):
        thr_dev = density_threshold.to(device=density_grid.device, dtype=_f32).reshape(1).contiguous()
        thr = 0.0
    else:
        thr = float(density_threshold)
    call("mfnerf_packbits", ptr(density_grid), density_bitfield.numel(), thr, ptr(thr_dev), ptr(density_bitfield),
         stream())


def _workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=_u8, device=device)


def raymarching_train(rays_o, rays_d, hits_t, density_bitfield, cascades, scale, exp_step_factor, noise,
                      grid_size, max_samples):
    """raymarching.cu:283-332.  Outputs sized N*max_samples as the reference (no zero-fill: only
    [0, counter[0]) is meaningful, which is all RayMarcher reads); rays_a rows in ray order."""
    for n, t, dt in (("rays_o", rays_o, _f32), ("rays_d", rays_d, _f32), ("hits_t", hits_t, _f32),
                     ("density_bitfield", density_bitfield, _u8), ("noise", noise, _f32)):
        check_input(n, t, dt)
    N = rays_o.shape[0]
    dev = rays_o.device
    cap = N * int(max_samples)
    rays_a = torch.empty(N, 3, dtype=_i64, device=dev)
    xyzs = torch.empty(cap, 3, dtype=_f32, device=dev)
    dirs = torch.empty(cap, 3, dtype=_f32, device=dev)
    deltas = torch.empty(cap, dtype=_f32, device=dev)
    ts = torch.empty(cap, dtype=_f32, device=dev)
    counter = torch.empty(2, dtype=_i32, device=dev)
    ws = _workspace(_lib_ws(N, int(max_samples)), dev)
    call("mfnerf_raymarching_train", ptr(rays_o), ptr(rays_d), ptr(hits_t), hits_t.stride(0), ptr(density_bitfield),
         int(cascades), float(scale), float(exp_step_factor), ptr(noise), int(grid_size), int(max_samples), N, cap,
         ptr(rays_a), ptr(xyzs), ptr(dirs), ptr(deltas), ptr(ts), ptr(counter), ptr(ws), stream())
    return [rays_a, xyzs, dirs, deltas, ts, counter]


def _lib_ws(n, max_samples):
    from ._lib import load
    return load().mfnerf_raymarching_train_workspace(n, max_samples)


def raymarching_test(rays_o, rays_d, hits_t, alive_indices, density_bitfield, cascades, scale, exp_step_factor,
                     grid_size, max_samples, N_samples):
    """raymarching.cu:407-454; hits_t is the (N,2) view hits_t[:,0] and is updated in place."""
    for n, t, dt in (("rays_o", rays_o, _f32), ("rays_d", rays_d, _f32), ("alive_indices", alive_indices, _i64),
                     ("density_bitfield", density_bitfield, _u8)):
        check_input(n, t, dt)
    if not hits_t.is_cuda or hits_t.dtype != _f32 or hits_t.dim() != 2 or hits_t.stride(1) != 1:
        raise RuntimeError("hits_t must be a CUDA float32 (N,2) row view")
    n = alive_indices.shape[0]
    dev = rays_o.device
    S = int(N_samples)
    xyzs = torch.empty(n, S, 3, dtype=_f32, device=dev)
    dirs = torch.empty(n, S, 3, dtype=_f32, device=dev)
    deltas = torch.empty(n, S, dtype=_f32, device=dev)
    ts = torch.empty(n, S, dtype=_f32, device=dev)
    n_eff = torch.empty(n, dtype=_i32, device=dev)
    call("mfnerf_raymarching_test", ptr(rays_o), ptr(rays_d), ptr(hits_t), hits_t.stride(0), ptr(alive_indices), n,
         ptr(density_bitfield), int(cascades), float(scale), float(exp_step_factor), int(grid_size),
         int(max_samples), S, ptr(xyzs), ptr(dirs), ptr(deltas), ptr(ts), ptr(n_eff), stream())
    return [xyzs, dirs, deltas, ts, n_eff]


def composite_train_fw(sigmas, rgbs, deltas, ts, rays_a, T_threshold):
    for n, t, dt in (("sigmas", sigmas, _f32), ("rgbs", rgbs, _f32), ("deltas", deltas, _f32), ("ts", ts, _f32),
                     ("rays_a", rays_a, _i64)):
        check_input(n, t, dt)
    N_rays, N = rays_a.shape[0], sigmas.shape[0]
    dev = sigmas.device
    opacity = torch.zeros(N_rays, dtype=_f32, device=dev)
    depth = torch.zeros(N_rays, dtype=_f32, device=dev)
    rgb = torch.zeros(N_rays, 3, dtype=_f32, device=dev)
    ws = torch.zeros(N, dtype=_f32, device=dev)
    total = torch.zeros(N_rays, dtype=_i64, device=dev)
    call("mfnerf_composite_train_fw", ptr(sigmas), ptr(rgbs), ptr(deltas), ptr(ts), ptr(rays_a), N_rays, N,
         float(T_threshold), ptr(total), ptr(opacity), ptr(depth), ptr(rgb), ptr(ws), stream())
    return [total, opacity, depth, rgb, ws]


def composite_train_bw(dL_dopacity, dL_ddepth, dL_drgb, dL_dws, sigmas, rgbs, ws, deltas, ts, rays_a, opacity,
                       depth, rgb, T_threshold):
    ins = (("dL_dopacity", dL_dopacity), ("dL_ddepth", dL_ddepth), ("dL_drgb", dL_drgb), ("dL_dws", dL_dws),
           ("sigmas", sigmas), ("rgbs", rgbs), ("ws", ws), ("deltas", deltas), ("ts", ts), ("opacity", opacity),
           ("depth", depth), ("rgb", rgb))
    for n, t in ins:
        check_input(n, t, _f32)
    check_input("rays_a", rays_a, _i64)
    N, N_rays = sigmas.shape[0], rays_a.shape[0]
    dev = sigmas.device
    dsig = torch.zeros(N, dtype=_f32, device=dev)
    drgb = torch.zeros(N, 3, dtype=_f32, device=dev)
    call("mfnerf_composite_train_bw", ptr(dL_dopacity), ptr(dL_ddepth), ptr(dL_drgb), ptr(dL_dws), ptr(sigmas),
         ptr(rgbs), ptr(ws), ptr(deltas), ptr(ts), ptr(rays_a), ptr(opacity), ptr(depth), ptr(rgb), N_rays, N,
         float(T_threshold), ptr(dsig), ptr(drgb), stream())
    return [dsig, drgb]


def composite_test_fw(sigmas, rgbs, deltas, ts, hits_t, alive_indices, T_threshold, N_eff_samples, opacity, depth,
                      rgb):
    for n, t, dt in (("sigmas", sigmas, _f32), ("rgbs", rgbs, _f32), ("deltas", deltas, _f32), ("ts", ts, _f32),
                     ("alive_indices", alive_indices, _i64), ("N_eff_samples", N_eff_samples, _i32),
                     ("opacity", opacity, _f32), ("depth", depth, _f32), ("rgb", rgb, _f32)):
        check_input(n, t, dt)
    n = alive_indices.shape[0]
    S = sigmas.shape[1] if sigmas.dim() == 2 else 0
    call("mfnerf_composite_test_fw", ptr(sigmas), ptr(rgbs), ptr(deltas), ptr(ts), ptr(alive_indices), n, S,
         float(T_threshold), ptr(N_eff_samples), ptr(opacity), ptr(depth), ptr(rgb), stream())


def distortion_loss_fw(ws, deltas, ts, rays_a):
    for n, t, dt in (("ws", ws, _f32), ("deltas", deltas, _f32), ("ts", ts, _f32), ("rays_a", rays_a, _i64)):
        check_input(n, t, dt)
    N_rays, N = rays_a.shape[0], ws.shape[0]
    dev = ws.device
    loss = torch.empty(N_rays, dtype=_f32, device=dev)
    wsi = torch.zeros(N, dtype=_f32, device=dev)
    wtsi = torch.zeros(N, dtype=_f32, device=dev)
    call("mfnerf_distortion_loss_fw", ptr(ws), ptr(deltas), ptr(ts), ptr(rays_a), N_rays, N, ptr(loss), ptr(wsi),
         ptr(wtsi), stream())
    return [loss, wsi, wtsi]


def distortion_loss_bw(dL_dloss, ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a):
    for n, t in (("dL_dloss", dL_dloss), ("ws_inclusive_scan", ws_inclusive_scan),
                 ("wts_inclusive_scan", wts_inclusive_scan), ("ws", ws), ("deltas", deltas), ("ts", ts)):
        check_input(n, t, _f32)
    check_input("rays_a", rays_a, _i64)
    N_rays, N = rays_a.shape[0], ws.shape[0]
    dws = torch.empty(N, dtype=_f32, device=ws.device)
    call("mfnerf_distortion_loss_bw", ptr(dL_dloss), ptr(ws_inclusive_scan), ptr(wts_inclusive_scan), ptr(ws),
         ptr(deltas), ptr(ts), ptr(rays_a), N_rays, N, ptr(dws), stream())
    return dws

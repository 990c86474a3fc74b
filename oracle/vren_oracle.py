"""oracle/vren_oracle.py -- TEST INFRASTRUCTURE ONLY (the parity checker).

A CPU `vren` module: the same 11 in-scope entry points, argument order and
return layout as the reference's pybind module (models/csrc/binding.cpp:234-250),
computed by the C restatement in oracle/vren_oracle.c on CPU torch tensors.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this.  It is also injected as `vren` into the reference's own Python
(tests/golden/make_golden.py) to produce the committed golden fixtures.
"""
import ctypes
import os
import subprocess

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_vren.so")
_lib = None

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int
_F = ctypes.c_float

_SIGS = {
    "orc_morton3D": [_I64, _P, _P],
    "orc_morton3D_invert": [_I64, _P, _P],
    "orc_packbits": [_I64, _P, _F, _P],
    "orc_ray_aabb_intersect": [_I64, _I64, _P, _P, _P, _P, _I, _P, _P, _P],
    "orc_raymarching_train": [_I64, _P, _P, _P, _P, _I, _F, _F, _P, _I, _I, _P, _P, _P, _P, _P, _P],
    "orc_raymarching_test": [_I64, _P, _P, _P, _P, _P, _I, _F, _F, _I, _I, _I, _P, _P, _P, _P, _P],
    "orc_composite_train_fw": [_I64, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _P],
    "orc_composite_train_bw": [_I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F, _P, _P, _P],
    "orc_composite_test_fw": [_I64, _I, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P],
    "orc_distortion_loss_fw": [_I64, _P, _P, _P, _P, _P, _P, _P],
    "orc_distortion_loss_bw": [_I64, _P, _P, _P, _P, _P, _P, _P, _P],
}


def build(force=False):
    """Compile the C restatement (contraction off, IEEE fp32) into oracle/liboracle_vren.so."""
    src = os.path.join(_HERE, "vren_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(_LIB_PATH)
        for name, argt in _SIGS.items():
            fn = getattr(_lib, name)
            fn.argtypes = argt
            fn.restype = None
    return _lib


def _chk(*ts):
    # models/csrc/include/utils.h:4-6 (CHECK_CONTIGUOUS); the oracle runs on CPU tensors.
    for t in ts:
        if not t.is_contiguous():
            raise RuntimeError("tensor must be contiguous")
        if t.is_cuda:
            raise RuntimeError("the oracle runs on CPU tensors")


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _f32(t):
    if t.dtype != torch.float32:
        raise RuntimeError(f"expected float32, got {t.dtype}")
    return t


def ray_aabb_intersect(rays_o, rays_d, centers, half_sizes, max_hits):
    """intersection.cu:59-100, including the host-side sort by t1 (:95-97)."""
    _chk(rays_o, rays_d, centers, half_sizes)
    N, V = rays_o.shape[0], centers.shape[0]
    hits_t = torch.zeros(N, max_hits, 2) - 1
    idx = torch.zeros(N, max_hits, dtype=torch.long) - 1
    cnt = torch.zeros(N, dtype=torch.int32)
    lib().orc_ray_aabb_intersect(N, V, _p(_f32(rays_o)), _p(_f32(rays_d)), _p(_f32(centers)),
                                 _p(_f32(half_sizes)), int(max_hits), _p(cnt), _p(hits_t), _p(idx))
    order = torch.sort(hits_t[..., 0])[1]
    idx = torch.gather(idx, 1, order)
    hits_t = torch.gather(hits_t, 1, order.unsqueeze(-1).tile((1, 1, 2)))
    return [cnt, hits_t, idx]


def morton3D(coords):
    _chk(coords)
    out = torch.zeros(coords.shape[0], dtype=coords.dtype)
    lib().orc_morton3D(coords.shape[0], _p(coords.int().contiguous()), _p(out))
    return out


def morton3D_invert(indices):
    _chk(indices)
    out = torch.zeros(indices.shape[0], 3, dtype=indices.dtype)
    lib().orc_morton3D_invert(indices.shape[0], _p(indices.int().contiguous()), _p(out))
    return out


def packbits(density_grid, density_threshold, density_bitfield):
    _chk(density_grid, density_bitfield)
    lib().orc_packbits(density_bitfield.shape[0], _p(_f32(density_grid)), float(density_threshold),
                       _p(density_bitfield))


def raymarching_train(rays_o, rays_d, hits_t, density_bitfield, cascades, scale, exp_step_factor,
                      noise, grid_size, max_samples):
    """raymarching.cu:283-332 (outputs sized N*max_samples as the reference; rows in ray order)."""
    _chk(rays_o, rays_d, hits_t, density_bitfield, noise)
    N = rays_o.shape[0]
    cap = N * max_samples
    rays_a = torch.zeros(N, 3, dtype=torch.long)
    xyzs = torch.zeros(cap, 3)
    dirs = torch.zeros(cap, 3)
    deltas = torch.zeros(cap)
    ts = torch.zeros(cap)
    counter = torch.zeros(2, dtype=torch.int32)
    lib().orc_raymarching_train(N, _p(_f32(rays_o)), _p(_f32(rays_d)), _p(_f32(hits_t).contiguous()),
                                _p(density_bitfield), int(cascades), float(scale), float(exp_step_factor),
                                _p(_f32(noise)), int(grid_size), int(max_samples),
                                _p(rays_a), _p(xyzs), _p(dirs), _p(deltas), _p(ts), _p(counter))
    return [rays_a, xyzs, dirs, deltas, ts, counter]


def raymarching_test(rays_o, rays_d, hits_t, alive_indices, density_bitfield, cascades, scale,
                     exp_step_factor, grid_size, max_samples, N_samples):
    """raymarching.cu:407-454.  `hits_t` (N,2) is updated in place (its [:,0] column)."""
    _chk(rays_o, rays_d, alive_indices, density_bitfield)
    n = alive_indices.shape[0]
    xyzs = torch.zeros(n, N_samples, 3)
    dirs = torch.zeros(n, N_samples, 3)
    deltas = torch.zeros(n, N_samples)
    ts = torch.zeros(n, N_samples)
    n_eff = torch.zeros(n, dtype=torch.int32)
    # the reference receives the strided view hits_t[:, 0] of the (N,1,2) tensor; the view is
    # row-contiguous with stride 2, which is exactly the (N,2) layout used here.
    if hits_t.dim() != 2 or hits_t.stride(1) != 1 or hits_t.stride(0) != 2:
        raise RuntimeError("hits_t must be an (N,2) row-major view")
    lib().orc_raymarching_test(n, _p(_f32(rays_o)), _p(_f32(rays_d)), _p(hits_t), _p(alive_indices),
                               _p(density_bitfield), int(cascades), float(scale), float(exp_step_factor),
                               int(grid_size), int(max_samples), int(N_samples),
                               _p(xyzs), _p(dirs), _p(deltas), _p(ts), _p(n_eff))
    return [xyzs, dirs, deltas, ts, n_eff]


def composite_train_fw(sigmas, rgbs, deltas, ts, rays_a, T_threshold):
    _chk(sigmas, rgbs, deltas, ts, rays_a)
    N_rays, N = rays_a.shape[0], sigmas.shape[0]
    opacity = torch.zeros(N_rays)
    depth = torch.zeros(N_rays)
    rgb = torch.zeros(N_rays, 3)
    ws = torch.zeros(N)
    total = torch.zeros(N_rays, dtype=torch.long)
    lib().orc_composite_train_fw(N_rays, _p(_f32(sigmas)), _p(_f32(rgbs)), _p(_f32(deltas)), _p(_f32(ts)),
                                 _p(rays_a), float(T_threshold), _p(total), _p(opacity), _p(depth),
                                 _p(rgb), _p(ws))
    return [total, opacity, depth, rgb, ws]


def composite_train_bw(dL_dopacity, dL_ddepth, dL_drgb, dL_dws, sigmas, rgbs, ws, deltas, ts, rays_a,
                       opacity, depth, rgb, T_threshold):
    ins = [dL_dopacity, dL_ddepth, dL_drgb, dL_dws, sigmas, rgbs, ws, deltas, ts, rays_a, opacity, depth, rgb]
    _chk(*ins)
    N, N_rays = sigmas.shape[0], rays_a.shape[0]
    dsig = torch.zeros(N)
    drgb = torch.zeros(N, 3)
    scratch = torch.zeros(max(N, 1))
    lib().orc_composite_train_bw(N_rays, *[_p(t) for t in ins[:9]], _p(rays_a), _p(opacity), _p(depth),
                                 _p(rgb), float(T_threshold), _p(scratch), _p(dsig), _p(drgb))
    return [dsig, drgb]


def composite_test_fw(sigmas, rgbs, deltas, ts, hits_t, alive_indices, T_threshold, N_eff_samples,
                      opacity, depth, rgb):
    _chk(sigmas, rgbs, deltas, ts, alive_indices, N_eff_samples, opacity, depth, rgb)
    n = alive_indices.shape[0]
    S = sigmas.shape[1] if sigmas.dim() == 2 else 0
    lib().orc_composite_test_fw(n, S, _p(_f32(sigmas)), _p(_f32(rgbs)), _p(_f32(deltas)), _p(_f32(ts)),
                                _p(alive_indices), float(T_threshold), _p(N_eff_samples), _p(opacity),
                                _p(depth), _p(rgb))


def distortion_loss_fw(ws, deltas, ts, rays_a):
    _chk(ws, deltas, ts, rays_a)
    N_rays, N = rays_a.shape[0], ws.shape[0]
    loss = torch.zeros(N_rays)
    wsi = torch.zeros(N)
    wtsi = torch.zeros(N)
    lib().orc_distortion_loss_fw(N_rays, _p(_f32(ws)), _p(_f32(deltas)), _p(_f32(ts)), _p(rays_a),
                                 _p(loss), _p(wsi), _p(wtsi))
    return [loss, wsi, wtsi]


def distortion_loss_bw(dL_dloss, ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a):
    _chk(dL_dloss, ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a)
    N_rays, N = rays_a.shape[0], ws.shape[0]
    dws = torch.zeros(N)
    lib().orc_distortion_loss_bw(N_rays, _p(_f32(dL_dloss)), _p(ws_inclusive_scan), _p(wts_inclusive_scan),
                                 _p(ws), _p(deltas), _p(ts), _p(rays_a), _p(dws))
    return dws

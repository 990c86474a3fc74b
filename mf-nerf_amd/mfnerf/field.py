"""Grid encoding and NGP field-head ops over the C ABI, plus their autograd Functions.

These replace the tiny-cuda-nn calls of models/networks.py:106,144-147 (xyz_encoder = HashGrid
or MixedFeature grid + FullyFusedMLP 32->64->16, dir_encoder = SH4, rgb_net = FullyFusedMLP
32->64->64->3 Sigmoid).  Parameter layout follows tcnn: xyz_encoder.params = [MLP (3072) |
grid table], rgb_net.params = (7168), every MLP layer a row-major (out, in) block.
"""
import math
import weakref

import torch

from ._lib import call, load, ptr, stream

XYZ_NET_PARAMS = 64 * 32 + 16 * 64


def rgb_net_params(width=64):
    return width * 32 + width * width + 16 * width


def grid_encode_fw(x, n, table16, layout, desc, x_min=0.0, x_range=1.0, n_dev=None, out=None):
    """x (>=n,3) f32 -> (n, L*F) f16 (rows beyond *n_dev untouched)."""
    if out is None:
        out = torch.empty(n, layout.L * layout.F, dtype=torch.float16, device=x.device)
    call("mfnerf_grid_encode_fw", ptr(x), int(n), ptr(n_dev), float(x_min), float(x_range), desc, ptr(table16),
         ptr(out), stream())
    return out


def grid_bw_workspace(desc, device):
    """Zeroed private-copy workspace for grid_encode_bw (stays zero between calls)."""
    nb = load().mfnerf_grid_encode_bw_workspace(desc)
    return torch.zeros(max(nb, 16) // 4, dtype=torch.float32, device=device)


def grid_bw_binned_workspace(desc, n, device):
    """Workspace of the partitioned scatter for up to n points (private copies zeroed)."""
    nb = load().mfnerf_grid_encode_bw_binned_workspace(desc, int(n))
    if nb < 0:
        raise RuntimeError("grid_encode_bw_binned: unsupported layout")
    return torch.zeros(max(nb, 16) // 4, dtype=torch.float32, device=device)


def grid_encode_bw(x, n, dL_dfeat, grad_table, layout, desc, x_min=0.0, x_range=1.0, n_dev=None, workspace=None,
                   fixed_point=False, binned=False, n_slots=0):
    """Accumulates into grad_table (float atomics); fixed_point=True: int32 fixed-point atomics with
    per-level scales from the L1 norm of dL_dfeat (grad_table must be zero; it is overwritten);
    binned=True (implies fixed point): the partitioned LDS scatter (workspace:
    grid_bw_binned_workspace(desc, n_slots or n); n_slots: the count its record slots are sized for)."""
    l1 = None
    if fixed_point or binned:
        l1 = torch.zeros(layout.L, dtype=torch.float32, device=x.device)
        call("mfnerf_grid_level_l1", ptr(dL_dfeat), int(n), ptr(n_dev), layout.L, ptr(l1), stream())
    if binned:
        call("mfnerf_grid_encode_bw_binned", ptr(x), int(n), ptr(n_dev), float(x_min), float(x_range), desc,
             ptr(dL_dfeat), ptr(grad_table), ptr(workspace), int(n_slots), ptr(l1), 3, stream())
        call("mfnerf_grid_encode_bw_finish", desc, ptr(grad_table), ptr(workspace), ptr(l1), stream())
        return
    call("mfnerf_grid_encode_bw", ptr(x), int(n), ptr(n_dev), float(x_min), float(x_range), desc, ptr(dL_dfeat),
         ptr(grad_table), ptr(workspace), ptr(l1), stream())


def pack_field_weights(params_xyz_net, params_rgb, rgb_width=64, out=None):
    nbytes = load().mfnerf_field_packed_bytes(rgb_width)
    if nbytes < 0:
        raise RuntimeError(f"rgb_width={rgb_width} is not supported by this build of the fused field head")
    if out is None:
        out = torch.empty(nbytes // 2, dtype=torch.float16, device=params_rgb.device)
    call("mfnerf_field_pack_weights", ptr(params_xyz_net), ptr(params_rgb), int(rgb_width), ptr(out), stream())
    return out


def field_fw(feat, dirs, n, packed, rgb_width=64, density_only=False, n_dev=None, sigma=None, rgb=None):
    dev = feat.device
    if sigma is None:
        sigma = torch.empty(n, dtype=torch.float32, device=dev)
    if rgb is None and not density_only:
        rgb = torch.empty(n, 3, dtype=torch.float32, device=dev)
    call("mfnerf_field_fw", ptr(feat), 0, ptr(dirs), int(n), ptr(n_dev), ptr(packed), int(rgb_width),
         int(bool(density_only)), ptr(sigma), ptr(rgb), stream())
    return sigma, rgb


def field_bw_workspace(n, rgb_width=64, device="cuda"):
    nb = load().mfnerf_field_bw_workspace(int(n), int(rgb_width))
    return torch.empty(nb // 4, dtype=torch.float32, device=device)


def field_bw(feat, dirs, n, packed, dL_dsigma, dL_drgb, grad_scale, dL_dfeat, grad_xyz_net, grad_rgb, workspace,
             rgb_width=64, n_dev=None, nonfinite=None):
    call("mfnerf_field_bw", ptr(feat), 0, ptr(dirs), int(n), ptr(n_dev), ptr(packed), int(rgb_width), ptr(dL_dsigma),
         ptr(dL_drgb), float(grad_scale), ptr(dL_dfeat), ptr(grad_xyz_net), ptr(grad_rgb), ptr(workspace),
         ptr(nonfinite), None, stream())


def pow2_grad_scale(max_abs):
    """Largest power of two keeping the largest incoming grad <= ~1 in the fp16 backward."""
    if not (max_abs > 0) or not math.isfinite(max_abs):
        return 1.0
    return float(2.0 ** max(0, min(24, math.floor(-math.log2(max_abs)))))


_ws_cache = {}


def _grid_ws(desc, device):
    """Per-(device, layout) private-copy workspace; every backward leaves it zero again."""
    key = (str(device), bytes(desc))
    if key not in _ws_cache:
        _ws_cache[key] = grid_bw_workspace(desc, device)
    return _ws_cache[key]


class GridEncodeFunction(torch.autograd.Function):
    """tcnn.Encoding(HashGrid/MixedFeatureGrid) forward/backward: x (N,3) in [0,1] -> (N, L*F) f16."""

    @staticmethod
    def forward(ctx, x, table, layout, desc):
        x = x.float().contiguous()
        feat = grid_encode_fw(x, x.shape[0], table.detach().half().contiguous(), layout, desc)
        ctx.save_for_backward(x)
        ctx.layout, ctx.desc, ctx.n_table = layout, desc, table.numel()
        return feat

    @staticmethod
    def backward(ctx, dL_dfeat):
        (x,) = ctx.saved_tensors
        g = torch.zeros(ctx.n_table, dtype=torch.float32, device=x.device)
        grid_encode_bw(x, x.shape[0], dL_dfeat.float().contiguous(), g, ctx.layout, ctx.desc,
                       workspace=_grid_ws(ctx.desc, x.device))
        return None, g, None, None


_weights_cache = {}


def field_weights(xyz_params, rgb_params, rgb_width):
    """(packed MLP fragments, fp16 table) of these parameter tensors, re-derived only when one of
    them changed (their version counters): the test-time loop calls the field many times per frame
    with the same weights."""
    key = (xyz_params.data_ptr(), rgb_params.data_ptr(), int(rgb_width))
    ver = (xyz_params._version, rgb_params._version)
    owners = tuple(p._base if p._base is not None else p for p in (xyz_params, rgb_params))
    hit = _weights_cache.get(key)
    # the owning tensors themselves (weakly held) must match: a new model whose parameters reuse a
    # freed model's memory and version counts must not be served the old weights
    if hit is not None and hit[0] == ver and all(r() is o for r, o in zip(hit[3], owners)):
        return hit[1], hit[2]
    net = xyz_params[:XYZ_NET_PARAMS].detach().contiguous()
    table16 = xyz_params[XYZ_NET_PARAMS:].detach().half().contiguous()
    packed = pack_field_weights(net, rgb_params.detach().contiguous(), rgb_width)
    _weights_cache.clear()  # the current model only
    _weights_cache[key] = (ver, packed, table16, tuple(weakref.ref(o) for o in owners))
    return packed, table16


class NGPFieldFunction(torch.autograd.Function):
    """Fused NGP.forward (networks.py:134-155): world xyz, dirs -> sigma f32 (N), rgb f32 (N,3).

    xyz_params = [xyz MLP (3072) | grid table]; rgb_params = rgb MLP.  The rgb values are fp16-
    representable (tcnn's half output), sigma = exp(h0) with h0 the fp16 network output."""

    @staticmethod
    def forward(ctx, xyzs, dirs, xyz_params, rgb_params, layout, desc, x_min, x_range, rgb_width):
        xyzs = xyzs.float().contiguous()
        dirs = dirs.float().contiguous()
        n = xyzs.shape[0]
        packed, table16 = field_weights(xyz_params, rgb_params, rgb_width)
        feat = grid_encode_fw(xyzs, n, table16, layout, desc, x_min, x_range)
        sigma, rgb = field_fw(feat, dirs, n, packed, rgb_width)
        ctx.save_for_backward(xyzs, dirs, feat, packed, sigma)
        ctx.cfg = (layout, desc, x_min, x_range, rgb_width, xyz_params.numel(), rgb_params.numel())
        return sigma, rgb

    @staticmethod
    def backward(ctx, dL_dsigma, dL_drgb):
        xyzs, dirs, feat, packed, sigma = ctx.saved_tensors
        layout, desc, x_min, x_range, rgb_width, n_xyz, n_rgb = ctx.cfg
        n = xyzs.shape[0]
        dev = xyzs.device
        dsig = torch.zeros(n, device=dev) if dL_dsigma is None else dL_dsigma.float().contiguous()
        drgb = torch.zeros(n, 3, device=dev) if dL_drgb is None else dL_drgb.float().contiguous()
        # a power-of-two scale for the fp16 MFMA backward, from the largest incoming gradient
        with torch.no_grad():
            m = torch.maximum(drgb.abs().max(), (dsig * sigma.clamp(max=3.3e6)).abs().max()) if n else \
                torch.zeros((), device=dev)
        S = pow2_grad_scale(float(m))
        g_xyz = torch.zeros(n_xyz, dtype=torch.float32, device=dev)
        g_rgb = torch.zeros(n_rgb, dtype=torch.float32, device=dev)
        dfeat = torch.empty(n, layout.L * layout.F, dtype=torch.float32, device=dev)
        ws = field_bw_workspace(n, rgb_width, dev)
        field_bw(feat, dirs, n, packed, dsig, drgb, S, dfeat, g_xyz[:XYZ_NET_PARAMS], g_rgb, ws, rgb_width)
        grid_encode_bw(xyzs, n, dfeat, g_xyz[XYZ_NET_PARAMS:], layout, desc, x_min, x_range,
                       workspace=_grid_ws(desc, dev))
        return None, None, g_xyz, g_rgb, None, None, None, None, None


class NGPDensityFunction(torch.autograd.Function):
    """NGP.density (networks.py:96-109) without the rgb head; forward only (used under no_grad)."""

    @staticmethod
    def forward(ctx, xyzs, xyz_params, rgb_params, layout, desc, x_min, x_range, rgb_width):
        xyzs = xyzs.float().contiguous()
        n = xyzs.shape[0]
        packed, table16 = field_weights(xyz_params, rgb_params, rgb_width)
        feat = grid_encode_fw(xyzs, n, table16, layout, desc, x_min, x_range)
        sigma, _ = field_fw(feat, None, n, packed, rgb_width, density_only=True)
        return sigma

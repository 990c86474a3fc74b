"""CPU tests: the oracle against known answers, host logic, and the C ABI library's exports.
No GPU compute here (the -m "not gpu" suite runs in the build container)."""
import ctypes
import math
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT
from mfnerf import synthetic

SQRT3 = 3 ** 0.5


def header_symbols():
    src = open(os.path.join(ROOT, "include", "mfnerf.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int64_t|int)\s+(mfnerf_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    from mfnerf import _lib
    assert os.path.exists(_lib.LIB_PATH), "build libmfnerf_hip.so first (__graft_entry__.build())"
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature"
    assert _lib.load().mfnerf_abi_version() == 2


def test_ops_reject_cpu_tensors_like_check_input():
    from mfnerf import vren
    with pytest.raises(RuntimeError, match="CUDA"):
        vren.morton3D(torch.zeros(4, 3, dtype=torch.int32))
    with pytest.raises(RuntimeError):
        vren.composite_train_fw(torch.zeros(4), torch.zeros(4, 3), torch.zeros(4), torch.zeros(4),
                                torch.zeros(1, 3, dtype=torch.long), 1e-4)


def test_morton_known_answers(oracle):
    c = torch.tensor([[1, 0, 0], [0, 1, 0], [0, 0, 1], [127, 127, 127], [3, 5, 6]], dtype=torch.int32)
    m = oracle.morton3D(c)
    assert m.tolist()[:4] == [1, 2, 4, 2 ** 21 - 1]
    assert torch.equal(oracle.morton3D_invert(m), c)


def test_packbits_matches_numpy(oracle):
    g = torch.Generator().manual_seed(0)
    grid = torch.randn(8 * 1000, generator=g)
    bf = torch.zeros(1000, dtype=torch.uint8)
    oracle.packbits(grid, 0.3, bf)
    assert torch.equal(bf, synthetic.packbits_np(grid, 0.3))


def test_composite_constant_sigma_closed_form(oracle):
    """w_k = (1 - e^{-s d}) e^{-k s d} until T <= thr (SURVEY.md 8c KAT 4)."""
    S, s, d = 40, 3.0, 0.01
    rays_a = torch.tensor([[0, 0, S]])
    sig = torch.full((S,), s)
    deltas = torch.full((S,), d)
    ts = torch.arange(S).float()
    rgbs = torch.rand(S, 3)
    tot, op, de, rgb, ws = oracle.composite_train_fw(sig, rgbs, deltas, ts, rays_a, 1e-4)
    a = 1 - math.exp(-s * d)
    w = torch.tensor([a * math.exp(-k * s * d) for k in range(S)])
    assert torch.allclose(ws, w.float(), rtol=1e-5)
    assert torch.allclose(op, w.sum().float().reshape(1), rtol=1e-5)
    assert tot.item() == S


def _composite_torch(sig, rgbs, deltas, ts, N):
    """Differentiable fp64 restatement (cumprod transmittance), no early stop."""
    a = 1 - torch.exp(-sig * deltas)
    T = torch.cumprod(torch.cat([torch.ones(1, dtype=a.dtype), 1 - a[:-1]]), 0)
    w = a * T
    return w.sum(), (w * ts).sum(), (w[:, None] * rgbs).sum(0), w


def test_composite_bw_matches_autograd(oracle):
    """composite_train_bw vs autograd of a cumprod restatement in fp64 (SURVEY.md 8c KAT 5)."""
    g = torch.Generator().manual_seed(1)
    S = 50
    sig = torch.rand(S, generator=g, dtype=torch.float64) * 20
    rgbs = torch.rand(S, 3, generator=g, dtype=torch.float64)
    deltas = torch.full((S,), 0.01, dtype=torch.float64)
    ts = torch.linspace(0.2, 1.0, S, dtype=torch.float64)
    dO, dD = torch.randn(1, generator=g, dtype=torch.float64), torch.randn(1, generator=g, dtype=torch.float64)
    dC, dW = torch.randn(1, 3, generator=g, dtype=torch.float64), torch.randn(S, generator=g, dtype=torch.float64)
    sv, cv = sig.clone().requires_grad_(True), rgbs.clone().requires_grad_(True)
    o, dpt, c, w = _composite_torch(sv, cv, deltas, ts, S)
    (o * dO[0] + dpt * dD[0] + (c * dC[0]).sum() + (w * dW).sum()).backward()
    f = lambda t: t.float().contiguous()  # noqa: E731
    rays_a = torch.tensor([[0, 0, S]])
    _, op, de, rgb, ws = oracle.composite_train_fw(f(sig), f(rgbs), f(deltas), f(ts), rays_a, 0.0)
    dsig, drgb = oracle.composite_train_bw(f(dO), f(dD), f(dC), f(dW), f(sig), f(rgbs), ws, f(deltas), f(ts),
                                           rays_a, op, de, rgb, 0.0)
    assert torch.allclose(dsig.double(), sv.grad, rtol=1e-3, atol=1e-5)
    assert torch.allclose(drgb.double(), cv.grad, rtol=1e-3, atol=1e-6)


def test_distortion_loss_definition(oracle):
    """O(n^2) definition: sum_ij w_i w_j |t_i - t_j| + 1/3 sum_i w_i^2 d_i (SURVEY.md 8c KAT 6)."""
    g = torch.Generator().manual_seed(2)
    S = 30
    ws = torch.rand(S, generator=g) * 0.1
    ts = torch.sort(torch.rand(S, generator=g))[0]
    deltas = torch.rand(S, generator=g) * 0.01
    loss, _, _ = oracle.distortion_loss_fw(ws, deltas, ts, torch.tensor([[0, 0, S]]))
    w, t, d = ws.double(), ts.double(), deltas.double()
    ref = (w[:, None] * w[None] * (t[:, None] - t[None]).abs()).sum() + (w * w * d).sum() / 3
    assert abs(loss.item() - ref.item()) < 1e-5 * max(1.0, ref.item())


def test_march_fully_occupied_closed_form(oracle):
    """Every hit ray gets samples t1 + noise*dt + k*dt < t2 (SURVEY.md 8c KAT 3)."""
    poses = synthetic.camera_poses(n_cams=5)
    o, d = synthetic.random_rays(300, poses, seed=4)
    _, ht, _ = oracle.ray_aabb_intersect(o, d, torch.zeros(1, 3), torch.full((1, 3), 0.5), 1)
    ht[(ht[:, 0, 0] >= 0) & (ht[:, 0, 0] < 0.01), 0, 0] = 0.01
    noise = torch.rand(300, generator=torch.Generator().manual_seed(5))
    full = torch.full((128 ** 3 // 8,), 255, dtype=torch.uint8)
    ra, x, dd, de, ts, cnt = oracle.raymarching_train(o, d, ht[:, 0].contiguous(), full, 1, 0.5, 0.0, noise, 128,
                                                      1024)
    dt = np.float32(SQRT3 / 1024)
    for r in range(300):
        t1, t2 = float(ht[r, 0, 0]), float(ht[r, 0, 1])
        n = int(ra[r, 2])
        if t1 < 0:
            assert n == 0
            continue
        t = np.float32(np.float32(dt) * np.float32(noise[r]) + np.float32(t1))
        k = 0
        while t < t2 and k < 1024:
            t = np.float32(t + dt)
            k += 1
        assert n == k
        s0 = int(ra[r, 1])
        assert torch.allclose(de[s0:s0 + n], torch.full((n,), float(dt)))


def test_grid_layout_sizing():
    from mfnerf.grid import GridLayout
    b = math.exp(math.log(2048 * 0.5 / 16) / 15)
    lay = GridLayout(16, 2, 19, 16, b)
    assert lay.res[:5] == [16, 22, 28, 37, 49]
    assert lay.n_params == 11445040  # fp32-faithful tcnn sizing, see DESIGN.md
    assert all(s <= 2 ** 19 for s in lay.sizes)
    mf = GridLayout(16, 2, 20, 16, b, "MixedFeature", 8)
    assert mf.n_params < lay.n_params and set(mf.kind) == {0, 1}


def test_grid_oracle_dense_level_is_trilinear():
    """A dense level holding a linear field f(g) = a.g reproduces a.(scale*x + 0.5) exactly
    away from the wrap-around face (SURVEY.md 8c KAT 7)."""
    from oracle import field_oracle as FO
    lay = FO.GridLayout(4, 2, 19, 16, 1.5)
    res = lay.res[1]
    n = lay.sizes[1]
    gi = torch.arange(n)
    gx, gy, gz = gi % res, (gi // res) % res, gi // (res * res)
    params = torch.zeros(lay.n_params)
    tab = params.view(-1, 2)
    tab[lay.offsets[1]:lay.offsets[1] + n, 0] = (1 * gx + 2 * gy + 3 * gz).float()
    x = torch.rand(500, 3) * 0.9
    out = FO.grid_encode(x, params, lay)[:, 2]
    pos = x * lay.scales[1] + 0.5
    assert torch.allclose(out, pos @ torch.tensor([1.0, 2.0, 3.0]), rtol=1e-5, atol=1e-4)

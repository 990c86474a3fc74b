"""GPU parity of the vren ops (mfnerf.vren -> libmfnerf_hip.so) against the CPU oracle.

Integer outputs (cell/Morton indices, sample counts, rays_a, marching sample positions, which
involve no transcendental) must match bit for bit; compositing floats to 1e-4 (north_star).
"""
import numpy as np
import pytest
import torch

from mfnerf import synthetic
from mfnerf import vren as V

pytestmark = pytest.mark.gpu

SQRT3 = 3 ** 0.5


def _to(d, *ts):
    return [t.to(d) for t in ts]


def lego_inputs(n_rays, seed=0, scale=0.5, cascades=1, exp_step=0.0):
    # real (unbounded) scenes: cameras inside the box, near the content (mip-NeRF 360 style)
    poses = synthetic.camera_poses(seed=seed, radius=1.5 if scale <= 0.5 else 2.0)
    o, d = synthetic.random_rays(n_rays, poses, seed=seed)
    grid = synthetic.ball_density_grid(cascades=cascades, scale=scale, seed=seed)
    bf = synthetic.packbits_np(grid, 0.01 * 1024 / SQRT3)
    return o, d, bf, grid


def aabb_hits(oracle, o, d, half=0.5):
    c = torch.zeros(1, 3)
    h = torch.full((1, 3), half)
    _, ht, _ = oracle.ray_aabb_intersect(o, d, c, h, 1)
    ht[(ht[:, 0, 0] >= 0) & (ht[:, 0, 0] < 0.01), 0, 0] = 0.01
    return ht


def test_morton_roundtrip_all_cells(gpu, oracle):
    G = 128
    r = torch.arange(G, dtype=torch.int32)
    c = torch.stack(torch.meshgrid(r, r, r, indexing="ij"), -1).reshape(-1, 3).contiguous()
    m_ref = oracle.morton3D(c)
    m = V.morton3D(c.to(gpu))
    assert torch.equal(m.cpu(), m_ref)
    inv = V.morton3D_invert(m)
    assert torch.equal(inv.cpu(), c)
    assert m_ref[1].item() == 4 and oracle.morton3D(torch.tensor([[1, 0, 0]], dtype=torch.int32)).item() == 1


def test_packbits(gpu, oracle):
    g = torch.Generator().manual_seed(1)
    grid = torch.randn(2, 128 ** 3, generator=g) * 4
    bf_ref = torch.zeros(2 * 128 ** 3 // 8, dtype=torch.uint8)
    oracle.packbits(grid, 0.7, bf_ref)
    bf = torch.zeros_like(bf_ref).to(gpu)
    V.packbits(grid.to(gpu), 0.7, bf)
    assert torch.equal(bf.cpu(), bf_ref)
    assert torch.equal(bf_ref, synthetic.packbits_np(grid, 0.7))
    bf2 = torch.zeros_like(bf_ref).to(gpu)
    V.packbits(grid.to(gpu), torch.tensor(0.7, device=gpu), bf2)  # device threshold (no host sync)
    assert torch.equal(bf2.cpu(), bf_ref)


@pytest.mark.parametrize("max_hits", [1, 3])
def test_ray_aabb_intersect(gpu, oracle, max_hits):
    g = torch.Generator().manual_seed(2)
    N = 4096
    o = (torch.rand(N, 3, generator=g) - 0.5) * 4
    d = torch.randn(N, 3, generator=g)
    d[:7, 1] = 0.0  # axis-parallel rays (inf inverse direction)
    V_ = 5 if max_hits > 1 else 1
    centers = (torch.rand(V_, 3, generator=g) - 0.5) * 1.5
    half = torch.rand(V_, 3, generator=g) * 0.4 + 0.1
    cnt_r, ht_r, idx_r = oracle.ray_aabb_intersect(o, d, centers, half, max_hits)
    cnt, ht, idx = V.ray_aabb_intersect(*_to(gpu, o, d, centers, half), max_hits)
    assert torch.equal(cnt.cpu(), cnt_r)
    if max_hits == 1:
        assert torch.equal(ht.cpu(), ht_r) and torch.equal(idx.cpu(), idx_r)
    else:  # ties in t1 may order differently; compare as sorted multisets per ray
        assert torch.equal(ht.cpu()[..., 0], ht_r[..., 0])
        key = lambda t, i: torch.sort(t[..., 1] + i.float() * 10, dim=1)[0]  # noqa: E731
        assert torch.allclose(key(ht.cpu(), idx.cpu()), key(ht_r, idx_r))


def _march_both(gpu, oracle, o, d, ht, bf, cascades, scale, exp_step, max_samples=1024, seed=3):
    noise = torch.rand(o.shape[0], generator=torch.Generator().manual_seed(seed))
    hits = ht[:, 0].contiguous()
    ref = oracle.raymarching_train(o, d, hits, bf, cascades, scale, exp_step, noise, 128, max_samples)
    out = V.raymarching_train(*_to(gpu, o, d, hits, bf), cascades, scale, exp_step, noise.to(gpu), 128, max_samples)
    return ref, [t.cpu() for t in out]


@pytest.mark.parametrize("n_rays", [1, 256, 1000, 8192, 12345])  # (ragged: the scan's partial batches)
def test_raymarching_train_lego_bitexact(gpu, oracle, n_rays):
    o, d, bf, _ = lego_inputs(n_rays)
    ht = aabb_hits(oracle, o, d)
    ref, out = _march_both(gpu, oracle, o, d, ht, bf, 1, 0.5, 0.0)
    ra_r, x_r, d_r, de_r, t_r, c_r = ref
    ra, x, dd, de, t, c = out
    assert torch.equal(c, c_r)
    assert torch.equal(ra, ra_r)
    n = int(c_r[0])
    for a, b in ((x, x_r), (dd, d_r), (de, de_r), (t, t_r)):
        assert torch.equal(a[:n], b[:n])
    if n_rays == 8192:
        assert 55 <= n / n_rays <= 70  # the calibrated Lego-like workload


def test_raymarching_train_real_scene_cascades(gpu, oracle):
    """garden-like config: scale 16 -> 6 cascades, exp_step 1/256 (benchmark_mipnerf360_mf.sh)."""
    scale = 16.0
    C = 6
    o, d, bf, _ = lego_inputs(2048, seed=5, scale=scale, cascades=C)
    ht = aabb_hits(oracle, o, d, half=scale)
    ref, out = _march_both(gpu, oracle, o, d, ht, bf, C, scale, 1 / 256)
    assert torch.equal(out[5], ref[5]) and torch.equal(out[0], ref[0])
    n = int(ref[5][0])
    assert n > 0
    for a, b in zip(out[1:5], ref[1:5]):
        assert torch.equal(a[:n], b[:n])


def test_raymarching_train_edges(gpu, oracle):
    o, d, bf, _ = lego_inputs(512, seed=7)
    ht = aabb_hits(oracle, o, d)
    ht[::5] = -1.0  # misses
    ref, out = _march_both(gpu, oracle, o, d, ht, bf, 1, 0.5, 0.0, max_samples=8)  # tight per-ray cap
    assert torch.equal(out[0], ref[0]) and torch.equal(out[5], ref[5])
    assert int(ref[0][::5, 2].sum()) == 0
    # fully occupied grid: closed-form counts t1+noise*dt + k*dt < t2
    full = torch.full_like(bf, 255)
    ref, out = _march_both(gpu, oracle, o, d, ht, full, 1, 0.5, 0.0)
    assert torch.equal(out[0], ref[0])
    dt = SQRT3 / 1024
    hit = ht[:, 0, 0] >= 0
    est = ((ht[:, 0, 1] - ht[:, 0, 0]) / dt).ceil()
    cnt = ref[0][:, 2].float()
    assert torch.all((cnt[hit] - est[hit]).abs() <= 1)


@pytest.mark.parametrize("N_samples", [1, 4, 64])
@pytest.mark.parametrize("exp_step", [0.0, 1 / 256])
def test_raymarching_test(gpu, oracle, N_samples, exp_step):
    C = 1 if exp_step == 0 else 2
    scale = 0.5 if exp_step == 0 else 1.0
    o, d, bf, _ = lego_inputs(2048, seed=11, scale=scale, cascades=C)
    ht = aabb_hits(oracle, o, d, half=scale)
    alive = torch.arange(0, 2048, 3, dtype=torch.long)
    ht_r = ht.clone()
    ref = oracle.raymarching_test(o, d, ht_r[:, 0], alive, bf, C, scale, exp_step, 128, 1024, N_samples)
    ht_g = ht.to(gpu)
    out = V.raymarching_test(*_to(gpu, o, d), ht_g[:, 0], alive.to(gpu), bf.to(gpu), C, scale, exp_step, 128, 1024,
                             N_samples)
    for a, b in zip(out, ref):
        assert torch.equal(a.cpu(), b)
    assert torch.equal(ht_g.cpu(), ht_r)  # in-place update of hits_t[:, 0]


def fixed64_batch(n_rays=2048, S=64, seed=1):
    """SURVEY.md 8d fixed-64 mode: rays_a[r] = (r, 64r, 64), sigma = exp(N(0,1.5^2))."""
    g = torch.Generator().manual_seed(seed)
    N = n_rays * S
    rays_a = torch.stack([torch.arange(n_rays), torch.arange(n_rays) * S, torch.full((n_rays,), S)], 1).long()
    sig = torch.exp(torch.randn(N, generator=g) * 1.5)
    rgbs = torch.rand(N, 3, generator=g)
    deltas = torch.full((N,), SQRT3 / 1024)
    ts = (torch.arange(N) % S).float() * (SQRT3 / 1024) + 0.3
    return rays_a, sig, rgbs, deltas, ts


def _ambiguous_rays(sig, deltas, rays_a, thr):
    """Rays whose transmittance passes within 1e-5 (relative) of T_threshold: their termination
    index may legitimately differ by one between expf and the hardware exp2."""
    amb = torch.zeros(rays_a.shape[0], dtype=torch.bool)
    for n in range(rays_a.shape[0]):
        s0, N = int(rays_a[n, 1]), int(rays_a[n, 2])
        T = torch.cumprod(torch.exp(-sig[s0:s0 + N].double() * deltas[s0:s0 + N].double()), 0)
        amb[n] = bool(((T / thr - 1).abs() < 1e-5).any())
    return amb


def test_composite_train_fw_bw(gpu, oracle):
    rays_a, sig, rgbs, deltas, ts = fixed64_batch()
    thr = 1e-4
    ref = oracle.composite_train_fw(sig, rgbs, deltas, ts, rays_a, thr)
    out = [t.cpu() for t in V.composite_train_fw(*_to(gpu, sig, rgbs, deltas, ts, rays_a), thr)]
    amb = _ambiguous_rays(sig, deltas, rays_a, thr)
    assert torch.equal(out[0][~amb], ref[0][~amb])
    for a, b in zip(out[1:], ref[1:]):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-5)
    g = torch.Generator().manual_seed(4)
    dO, dD = torch.randn(2048, generator=g), torch.randn(2048, generator=g)
    dC, dW = torch.randn(2048, 3, generator=g), torch.randn(sig.shape[0], generator=g)
    _, op, de, rgb, ws = ref
    ref_b = oracle.composite_train_bw(dO, dD, dC, dW, sig, rgbs, ws, deltas, ts, rays_a, op, de, rgb, thr)
    out_b = V.composite_train_bw(*_to(gpu, dO, dD, dC, dW, sig, rgbs, ws, deltas, ts, rays_a, op, de, rgb), thr)
    for a, b in zip(out_b, ref_b):
        assert torch.allclose(a.cpu(), b, rtol=1e-4, atol=1e-4 * float(b.abs().max()))


def test_composite_train_on_marched_lego(gpu, oracle):
    o, d, bf, _ = lego_inputs(4096, seed=9)
    ht = aabb_hits(oracle, o, d)
    ref, _ = _march_both(gpu, oracle, o, d, ht, bf, 1, 0.5, 0.0)
    rays_a, _, _, deltas, ts, cnt = ref
    n = int(cnt[0])
    g = torch.Generator().manual_seed(8)
    sig = torch.exp(torch.randn(n, generator=g) * 2)
    rgbs = torch.rand(n, 3, generator=g)
    deltas, ts = deltas[:n].contiguous(), ts[:n].contiguous()
    r = oracle.composite_train_fw(sig, rgbs, deltas, ts, rays_a, 1e-4)
    o_ = [t.cpu() for t in V.composite_train_fw(*_to(gpu, sig, rgbs, deltas, ts, rays_a), 1e-4)]
    amb = _ambiguous_rays(sig, deltas, rays_a, 1e-4)
    assert torch.equal(o_[0][~amb], r[0][~amb])
    for a, b in zip(o_[1:], r[1:]):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-5)


def test_composite_test_fw(gpu, oracle):
    g = torch.Generator().manual_seed(12)
    n, S, Nr = 1500, 8, 3000
    alive = torch.randperm(Nr, generator=g)[:n].long()
    sig = torch.exp(torch.randn(n, S, generator=g) * 2)
    rgbs = torch.rand(n, S, 3, generator=g)
    deltas = torch.full((n, S), SQRT3 / 1024)
    ts = torch.rand(n, S, generator=g)
    n_eff = torch.randint(0, S + 1, (n,), generator=g, dtype=torch.int32)
    op = torch.rand(Nr, generator=g) * 0.5
    de, rgb = torch.rand(Nr, generator=g), torch.rand(Nr, 3, generator=g)
    ar, opr, der, rgbr = alive.clone(), op.clone(), de.clone(), rgb.clone()
    oracle.composite_test_fw(sig, rgbs, deltas, ts, None, ar, 1e-4, n_eff, opr, der, rgbr)
    ag, opg, deg, rgbg = _to(gpu, alive, op, de, rgb)
    V.composite_test_fw(*_to(gpu, sig, rgbs, deltas, ts), None, ag, 1e-4, n_eff.to(gpu), opg, deg, rgbg)
    assert torch.equal(ag.cpu(), ar)
    for a, b in ((opg, opr), (deg, der), (rgbg, rgbr)):
        assert torch.allclose(a.cpu(), b, rtol=1e-4, atol=1e-5)


def test_distortion_loss(gpu, oracle):
    rays_a, sig, rgbs, deltas, ts = fixed64_batch(512, 32, seed=5)
    ws = torch.rand(sig.shape[0], generator=torch.Generator().manual_seed(6)) * 0.1
    rays_a[7, 2] = 0  # an empty ray
    ref = oracle.distortion_loss_fw(ws, deltas, ts, rays_a)
    out = V.distortion_loss_fw(*_to(gpu, ws, deltas, ts, rays_a))
    for a, b in zip(out, ref):
        assert torch.allclose(a.cpu(), b, rtol=1e-4, atol=1e-6)
    dl = torch.randn(512, generator=torch.Generator().manual_seed(7))
    rb = oracle.distortion_loss_bw(dl, ref[1], ref[2], ws, deltas, ts, rays_a)
    ob = V.distortion_loss_bw(*_to(gpu, dl, ref[1], ref[2], ws, deltas, ts, rays_a))
    assert torch.allclose(ob.cpu(), rb, rtol=1e-4, atol=1e-6)


def test_errors_like_check_input(gpu):
    with pytest.raises(RuntimeError):
        V.morton3D(torch.zeros(4, 3, dtype=torch.int32))  # CPU tensor
    with pytest.raises(RuntimeError):
        V.morton3D(torch.zeros(3, 4, dtype=torch.int32, device=gpu).t())  # non-contiguous


def _fused_vs_separate(gpu, oracle, rays_a, sig, rgbs, deltas, ts, seed=0, lam=1e-3):
    """mfnerf_composite_train_fused against the three separate launches (bit for bit) and the
    oracle's fw/bw driven by the loss gradient (1e-4)."""
    from mfnerf._lib import call, ptr, stream
    thr, n_rays, n = 1e-4, rays_a.shape[0], sig.shape[0]
    g = torch.Generator().manual_seed(seed)
    target = torch.rand(n_rays, 3, generator=g)
    S, C, Dt, Tt, R, T = _to(gpu, sig, rgbs, deltas, ts, rays_a, target)
    f32 = dict(dtype=torch.float32, device=gpu)

    def outs():
        return dict(total=torch.zeros(n_rays, dtype=torch.int64, device=gpu), op=torch.zeros(n_rays, **f32),
                    de=torch.zeros(n_rays, **f32), rgb=torch.zeros(n_rays, 3, **f32), ws=torch.zeros(n, **f32),
                    g_rgb=torch.zeros(n_rays, 3, **f32), g_op=torch.zeros(n_rays, **f32),
                    dsig=torch.zeros(n, **f32), drgb=torch.zeros(n, 3, **f32),
                    loss=torch.zeros(max(64, (n_rays + 3) // 4), **f32))
    a, b = outs(), outs()
    call("mfnerf_composite_train_fused", ptr(S), ptr(C), ptr(Dt), ptr(Tt), ptr(R), n_rays, n, thr, ptr(T), n_rays, lam,
         1.0, 1.0, 1.0, ptr(a["total"]), ptr(a["op"]), ptr(a["de"]), ptr(a["rgb"]), ptr(a["ws"]), ptr(a["g_rgb"]),
         ptr(a["g_op"]), ptr(a["dsig"]), ptr(a["drgb"]), ptr(a["loss"]), stream())
    call("mfnerf_composite_train_fw", ptr(S), ptr(C), ptr(Dt), ptr(Tt), ptr(R), n_rays, n, thr, ptr(b["total"]),
         ptr(b["op"]), ptr(b["de"]), ptr(b["rgb"]), ptr(b["ws"]), stream())
    call("mfnerf_nerf_loss", ptr(b["rgb"]), ptr(b["op"]), ptr(T), n_rays, n_rays, lam, 1.0, 1.0, 1.0,
         ptr(b["g_rgb"]), ptr(b["g_op"]), ptr(b["loss"]), stream())
    zr, zs = torch.zeros(n_rays, **f32), torch.zeros(n, **f32)
    call("mfnerf_composite_train_bw", ptr(b["g_op"]), ptr(zr), ptr(b["g_rgb"]), ptr(zs), ptr(S), ptr(C),
         ptr(b["ws"]), ptr(Dt), ptr(Tt), ptr(R), ptr(b["op"]), ptr(b["de"]), ptr(b["rgb"]), n_rays, n, thr,
         ptr(b["dsig"]), ptr(b["drgb"]), stream())
    torch.cuda.synchronize()
    for k in a:
        if k == "loss":
            assert abs(float(a[k].sum()) - float(b[k].sum())) <= 1e-6 * abs(float(b[k].sum()))
        else:
            assert torch.equal(a[k], b[k]), k
    # the oracle, driven by the same loss gradient
    ref = oracle.composite_train_fw(sig, rgbs, deltas, ts, rays_a, thr)
    amb = _ambiguous_rays(sig, deltas, rays_a, thr)
    assert torch.equal(a["total"].cpu()[~amb], ref[0][~amb])
    _, op, de, rgb, ws = ref
    g_rgb, g_op = a["g_rgb"].cpu(), a["g_op"].cpu()
    ref_b = oracle.composite_train_bw(g_op, torch.zeros(n_rays), g_rgb, torch.zeros(n), sig, rgbs, ws, deltas, ts,
                                      rays_a, op, de, rgb, thr)
    keep = ~amb[torch.repeat_interleave(torch.arange(n_rays), rays_a[:, 2])] if n == int(rays_a[:, 2].sum()) else None
    for got, want in zip((a["dsig"].cpu(), a["drgb"].cpu()), ref_b):
        if keep is not None:
            got, want = got[keep], want[keep]
        assert torch.allclose(got, want, rtol=1e-4, atol=1e-4 * float(want.abs().max()))


def test_composite_train_fused_fixed64(gpu, oracle):
    rays_a, sig, rgbs, deltas, ts = fixed64_batch()
    _fused_vs_separate(gpu, oracle, rays_a, sig, rgbs, deltas, ts)


def test_composite_train_fused_on_marched_lego(gpu, oracle):
    """Variable-length rays (many beyond one 64-sample chunk), misses (0 samples) included."""
    o, d, bf, _ = lego_inputs(4096, seed=9)
    ht = aabb_hits(oracle, o, d)
    ref, _ = _march_both(gpu, oracle, o, d, ht, bf, 1, 0.5, 0.0)
    rays_a, _, _, deltas, ts, cnt = ref
    n = int(cnt[0])
    assert int(rays_a[:, 2].max()) > 128 and int((rays_a[:, 2] == 0).sum()) > 0
    g = torch.Generator().manual_seed(8)
    sig = torch.exp(torch.randn(n, generator=g) * 2)
    rgbs = torch.rand(n, 3, generator=g)
    _fused_vs_separate(gpu, oracle, rays_a, sig, rgbs, deltas[:n].contiguous(), ts[:n].contiguous(), seed=3)

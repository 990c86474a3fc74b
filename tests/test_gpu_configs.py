"""BASELINE configs 3 and 4 at full size through the fused training step (TrainStep), stage by stage
against the oracles on the step's own intermediates:

* config 3 -- Synthetic-NeRF MixedFeature (benchmark_synthetic_nerf_mf.sh): 8 tables, T 2^20,
  rgb 128x2, 16384 rays, lr 2e-2, bounded (scale 0.5, 1 cascade, white background);
* config 4 -- mip-NeRF360 garden (benchmark_mipnerf360_mf.sh:28-33): scale 16 -> 6 cascades,
  exp-step 1/256, black background, MixedFeature 8 tables at T 2^20 and 2^22, rgb 128x2,
  4096 rays, lr 2e-2.

Per step: the march bit-exact vs raymarching.cu (oracle) on the whole batch; the encoding and the
field head on a seeded sample subset vs oracle/field_oracle.py; compositing + NeRFLoss forward and
backward on the whole batch vs volumerendering.cu (oracle) and losses.py restated; dL/dfeat on the
subset; the MLP weight gradients and the fixed-point table gradient (partitioned scatter) on the
whole batch vs the oracle's sums in fp32 / fp64; then three finite Adam steps.  The scenes are
synthetic (no datasets in this image): a ball union for config 3, and for config 4 a central object
inside a shell of background balls out to |x| ~ 14 (the unbounded cascades' range)."""
import math

import numpy as np
import pytest
import torch

from mfnerf import engine, synthetic
from mfnerf.field import XYZ_NET_PARAMS
from oracle import field_oracle as FO

pytestmark = pytest.mark.gpu

SUBSET = 8192


def _garden_grid(cascades, scale, seed=0):
    g = np.random.default_rng(seed)
    centers = [np.zeros(3)]
    radii = [0.35]
    for _ in range(160):  # background: a shell of balls at distance 1.5 .. 14
        v = g.normal(size=3)
        v /= np.linalg.norm(v)
        r = g.uniform(1.5, 14.0)
        centers.append(v * r)
        radii.append(g.uniform(0.06, 0.12) * r)
    return synthetic.balls_to_grid(np.array(centers), np.array(radii), cascades=cascades, scale=scale)


CONFIGS = {
    "config3-synthetic-mf-T20": (dict(n_rays=16384, grid="MixedFeature", N_tables=8, log2_T=20, rgb_width=128,
                                      lr=2e-2), "balls"),
    "config4-garden-mf-T20": (dict(n_rays=4096, scale=16.0, grid="MixedFeature", N_tables=8, log2_T=20,
                                   rgb_width=128, lr=2e-2), "garden"),
    "config4-garden-mf-T22": (dict(n_rays=4096, scale=16.0, grid="MixedFeature", N_tables=8, log2_T=22,
                                   rgb_width=128, lr=2e-2), "garden"),
}


def _batch(st, scene, seed):
    n = st.cfg.n_rays
    if scene == "balls":
        o, d = synthetic.random_rays(n, synthetic.camera_poses(seed=seed), seed=seed)
    else:  # cameras on a ring around the object, looking at it (the 360 captures' geometry)
        o, d = synthetic.random_rays(n, synthetic.camera_poses(radius=1.2, seed=seed), seed=seed, W=311, H=207,
                                     focal=240.0)
        d = d / d.norm(dim=1, keepdim=True)  # ray_utils.get_rays normalises (colmap)
    rgb = torch.rand(n, 3, generator=torch.Generator().manual_seed(seed + 99))
    return engine.Batch(o.to(st.dev), d.contiguous().to(st.dev), rgb.to(st.dev))


def _olayout(st):
    c = st.cfg
    b = float(np.exp(np.log(c.N_max * c.scale / c.N_min) / (c.L - 1)))
    return FO.GridLayout(c.L, c.F, c.log2_T, c.N_min, b, c.grid, c.N_tables)


@pytest.mark.parametrize("name", list(CONFIGS))
def test_config_full_size_step_vs_oracle(gpu, oracle, name):
    kw, scene = CONFIGS[name]
    cfg = engine.StepConfig(**kw)
    st = engine.TrainStep(cfg, device=gpu, seed=0)
    assert st.cascades == (1 if scene == "balls" else 6)
    grid = synthetic.ball_density_grid() if scene == "balls" else _garden_grid(st.cascades, cfg.scale)
    st.set_occupancy(grid)
    batch = _batch(st, scene, seed=11)
    st.run(batch, optimize=False)
    torch.cuda.synchronize()
    cpu = lambda t: t.detach().float().cpu() if t.is_floating_point() else t.detach().cpu()  # noqa: E731

    # --- march: bit-exact vs the oracle on the whole batch (raymarching.cu:166-280)
    rays_a, xyzs, dirs, deltas, ts = [cpu(t) for t in st.gather_march()]
    n = xyzs.shape[0]
    o, d = cpu(batch.rays_o), cpu(batch.rays_d)
    c, h = torch.zeros(1, 3), torch.full((1, 3), cfg.scale)
    _, ht, _ = oracle.ray_aabb_intersect(o, d, c, h, 1)
    t1 = ht[:, 0, 0]
    t1[(t1 >= 0) & (t1 < engine.NEAR_DISTANCE)] = engine.NEAR_DISTANCE
    exp_step = 0.0 if cfg.scale <= 0.5 else 1 / 256
    ref = oracle.raymarching_train(o, d, ht[:, 0].contiguous(), cpu(st.bitfield), st.cascades, cfg.scale, exp_step,
                                   cpu(st.state.noise), st.G, cfg.max_samples)
    n_o = int(ref[5][0])
    assert n == n_o and n > 20 * cfg.n_rays, (n, n_o)
    assert torch.equal(rays_a, ref[0])
    for got, want in zip((xyzs, dirs, deltas, ts), ref[1:5]):
        assert torch.equal(got, want[:n])
    if scene == "garden":  # the outer cascades are really marched (exp-step, beyond the unit cube)
        assert float(xyzs.abs().max()) > 4.0

    # --- the step's parameters as the oracle sees them (fp16 copies the kernels read)
    p = cpu(st.params)
    px, pr = p[:XYZ_NET_PARAMS], p[st.off_rgb:st.off_table]
    table16 = p[st.off_table:st.n_params].half().float()
    olay = _olayout(st)
    t = st.parts[0]
    g = torch.Generator().manual_seed(5)
    idx = torch.randperm(n, generator=g)[:SUBSET]
    xn = (xyzs[idx] - st.x_min) / st.x_range  # networks.py:105

    # --- encoding on the subset (planar (L, cap, F) half2 planes)
    feat = t.feat[:, :n].permute(1, 0, 2).reshape(n, cfg.L * cfg.F)
    feat_s = cpu(feat[idx.to(gpu)])
    enc_ref = FO.grid_encode(xn, table16, olay)
    assert torch.allclose(feat_s, enc_ref, atol=1e-3, rtol=0)

    # --- field head forward on the subset, from the kernels' own features
    sig_ref, rgb_ref, acts = FO.ngp_field_fw16(feat_s.half(), dirs[idx], px, pr, cfg.rgb_width)
    sig, rgb_s = cpu(t.sigma[:n]), cpu(t.rgb_s[:n])
    assert torch.allclose(sig[idx], sig_ref, rtol=4e-3, atol=1e-6)
    assert torch.allclose(rgb_s[idx], rgb_ref, atol=2e-3, rtol=0)

    # --- compositing + NeRFLoss on the whole batch (volumerendering.cu, losses.py:47-60,
    #     rendering.py:153-161 background), from the kernels' sigma / rgb
    total, op, depth, rgb, ws = oracle.composite_train_fw(sig, rgb_s, deltas, ts, rays_a, cfg.T_threshold)
    assert torch.equal(cpu(t.total), total)
    for got, want in ((t.opacity, op), (t.depth, depth), (t.rgb, rgb), (t.ws[:n], ws)):
        assert torch.allclose(cpu(got), want, rtol=1e-4, atol=1e-5)
    bg = 1.0 if cfg.scale <= 0.5 else 0.0
    target = cpu(batch.rgb)
    pred = rgb + bg * (1 - op[:, None])
    oo = op + 1e-10
    loss = float(((pred - target) ** 2).mean() + cfg.lambda_opacity * (-oo * torch.log(oo)).mean())
    assert abs(float(st.loss_sum) - loss) <= 1e-4 * loss, (float(st.loss_sum), loss)
    N = cfg.n_rays
    dL_dpred = 2 * (pred - target) / (3 * N)
    dL_dop = -bg * dL_dpred.sum(1) + cfg.lambda_opacity * (-torch.log(oo) - 1) / N
    dsig_ref, drgb_ref = oracle.composite_train_bw(dL_dop, torch.zeros(N), dL_dpred, torch.zeros(n), sig, rgb_s, ws,
                                                   deltas, ts, rays_a, op, depth, rgb, cfg.T_threshold)
    dsig, drgb = cpu(t.dsig[:n]), cpu(t.drgb_s[:n])
    assert torch.allclose(dsig, dsig_ref, rtol=1e-3, atol=1e-4 * float(dsig_ref.abs().max()))
    assert torch.allclose(drgb, drgb_ref, rtol=1e-3, atol=1e-4 * float(drgb_ref.abs().max()))

    # --- field backward: dL/dfeat on the subset (fp16-point emulation, the step's loss scale)
    S = st.loss_scale()
    dfeat_ref = FO.ngp_field_bw16(acts, dsig[idx], drgb[idx], S)[0]
    dfeat = cpu(t.dfeat[:n])
    err = float((dfeat[idx] - dfeat_ref).abs().max() / dfeat_ref.abs().max())
    assert err < 2e-3, err

    # --- the MLP weight gradients, summed over the whole batch (oracle in chunks)
    gx = torch.zeros(XYZ_NET_PARAMS)
    gr = torch.zeros(st.off_table - st.off_rgb)
    for a in range(0, n, 131072):
        f16 = feat[a:a + 131072].cpu()
        _, _, ac = FO.ngp_field_fw16(f16, dirs[a:a + 131072], px, pr, cfg.rgb_width)
        _, dx, dr = FO.ngp_field_bw16(ac, dsig[a:a + 131072], drgb[a:a + 131072], S)
        gx += dx
        gr += dr
    grads = cpu(st.grads)
    for got, want in ((grads[:XYZ_NET_PARAMS], gx), (grads[st.off_rgb:st.off_table], gr)):
        e = float((got - want).abs().max() / want.abs().max())
        assert e < 5e-3, e

    # --- the table gradient (int32 fixed point, partitioned scatter) vs fp64 sums of the same
    #     dL/dfeat over every sample, per table (MixedFeature levels share tables)
    #     (hashed levels: each contribution an fp16 record value, within 2^-11 of the sum of the
    #     entry's |contributions|, see test_gpu_field.REC_REL)
    tp = torch.zeros(olay.n_params, dtype=torch.float64).requires_grad_(True)
    ta = torch.zeros(olay.n_params, dtype=torch.float64).requires_grad_(True)
    xall = (xyzs - st.x_min) / st.x_range
    for a in range(0, n, 262144):
        enc = FO.grid_encode(xall[a:a + 262144], tp, olay)
        (enc * dfeat[a:a + 262144].double()).sum().backward()
        (FO.grid_encode(xall[a:a + 262144], ta, olay) * dfeat[a:a + 262144].abs().double()).sum().backward()
    gref, gabs = tp.grad, ta.grad
    gt = grads[st.off_table:st.n_params].double()
    regions = sorted({(olay.offsets[l], olay.sizes[l]) for l in range(cfg.L)})
    for off, size in regions:
        a, b = 2 * off, 2 * (off + size)
        scale = float(gref[a:b].abs().max())
        assert scale > 0
        excess = (gt[a:b] - gref[a:b]).abs() - (2.0 ** -11 * 1.0001 * gabs[a:b] + 1e-3 * scale)
        assert float(excess.max()) <= 0, (off, float(excess.max()) / scale)

    # --- three optimizer steps: finite, none skipped, the parameters move
    p0 = st.params.clone()
    for k in range(3):
        st.run(_batch(st, scene, seed=20 + k))
    torch.cuda.synchronize()
    assert st.skipped_steps() == 0 and math.isfinite(float(st.loss_sum))
    assert bool(torch.isfinite(st.params).all()) and not torch.equal(st.params, p0)
    assert int(st.step_dev) == 3

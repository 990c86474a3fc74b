"""Training harness on the GPU: device batch sampling (base.py:22-35 + get_rays), the GradScaler
skip on non-finite gradients, checkpoints in the reference's key layout, and an end-to-end run
(occupancy cadence, cosine LR, pipelined graphs, test-time renderer) that must learn a scene."""
import math

import pytest
import torch

from mfnerf import data, engine, synthetic
from mfnerf.trainer import HParams, Trainer

pytestmark = pytest.mark.gpu


def test_sample_rays_matches_torch(gpu):
    g = torch.Generator().manual_seed(0)
    n_img, hw, N = 5, 300, 4096
    imgs, poses, dirs = torch.rand(n_img, hw, 3, generator=g), torch.randn(n_img, 3, 4, generator=g), \
        torch.randn(hw, 3, generator=g)
    ds = data.DeviceDataset(imgs, poses, dirs, device=gpu, seed=3)
    out = torch.empty(3, N, 3, device=gpu)
    ii, pp = torch.empty(N, dtype=torch.int32, device=gpu), torch.empty(N, dtype=torch.int32, device=gpu)
    ds.sample(out, ii, pp)
    oc, ic, pc = out.cpu(), ii.cpu().long(), pp.cpu().long()
    assert torch.equal(oc[2], imgs[ic, pc])
    o, d = data.get_rays(dirs[pc], poses[ic])
    assert torch.equal(oc[0], o) and torch.allclose(oc[1], d, atol=1e-5)
    assert set(ic.tolist()) == set(range(n_img)) and len(set(pc.tolist())) > 0.9 * hw
    # the device counter advances: a second draw differs; same_image draws one image per batch
    out2 = torch.empty(3, N, 3, device=gpu)
    ds.sample(out2)
    assert not torch.equal(out2.cpu(), oc)
    same = data.DeviceDataset(imgs, poses, dirs, device=gpu, strategy="same_image")
    same.sample(out, ii, pp)
    assert len(set(ii.cpu().tolist())) == 1


def test_sample_rays_batches_are_independent(gpu):
    """Consecutive draws share no structure: over 1e8 (image, pixel) pairs, batches c, c+1, c+2
    have ~0 pairs in common (a counter hash with the call added linearly made batch c+2 batch c
    shifted by one ray -- the model then trains on two alternating batches)."""
    n_img, hw, N = 1000, 100000, 4096
    ds = data.DeviceDataset(torch.zeros(n_img, hw, 3), torch.zeros(n_img, 3, 4), torch.zeros(hw, 3), device=gpu)
    out = torch.empty(3, N, 3, device=gpu)
    ii, pp = torch.empty(N, dtype=torch.int32, device=gpu), torch.empty(N, dtype=torch.int32, device=gpu)
    sets = []
    for _ in range(4):
        ds.sample(out, ii, pp)
        sets.append(set((ii.long() * hw + pp.long()).cpu().tolist()))
    for a in range(4):
        for b in range(a + 1, 4):
            assert len(sets[a] & sets[b]) < 10, (a, b, len(sets[a] & sets[b]))


def test_nonfinite_gradient_skips_the_step(gpu):
    """GradScaler semantics (PL precision=16, train.py:287): a step whose gradient holds an inf/nan
    changes no parameter, no Adam moment and no step count; it is counted as skipped and leaves the
    gradient zero for the next step.  The NaN enters through the loss target, so the flag is the one
    the step itself raises (field_bw's dL/dfeat and weight-gradient checks), not a gradient scan."""
    st = engine.TrainStep(engine.StepConfig(n_rays=256, log2_T=14), device=gpu)
    st.set_occupancy(synthetic.ball_density_grid())
    bad, good = st.make_batches(2, seed=3)
    bad.rgb.fill_(float("nan"))
    p0, m0, s0 = st.params.clone(), st.m.clone(), int(st.step_dev)
    st.run(bad)
    torch.cuda.synchronize()
    assert torch.equal(st.params, p0) and torch.equal(st.m, m0) and int(st.step_dev) == s0
    assert st.skipped_steps() == 1 and int(st.finite_status[0]) == 0
    assert int((st.grads != 0).sum()) == 0  # zeroed for the next step even though skipped
    st.run(good)
    torch.cuda.synchronize()
    assert not torch.equal(st.params, p0) and int(st.step_dev) == s0 + 1 and st.skipped_steps() == 1
    assert torch.isfinite(st.params).all()


def _ball_views(n, W=64, seed=0):
    focal = 0.5 * W / math.tan(0.5 * 0.6911112)  # the Lego field of view
    return data.ball_scene_views(data.BallScene(n_balls=6, seed=1), n, W, focal, seed=seed)


def test_trainer_learns_a_scene_and_checkpoints(gpu, tmp_path):
    imgs, poses, dirs, K = _ball_views(100)
    t_imgs, t_poses, _, _ = _ball_views(4, seed=7)
    ds = data.DeviceDataset(imgs, poses, dirs, K=K, img_wh=(64, 64), device=gpu, seed=5)
    hp = HParams(batch_size=4096, T=16, num_epochs=2, steps_per_epoch=600)
    tr = Trainer(hp, ds, device=gpu)
    hist = tr.fit(log_every=200)
    psnr, per_view = tr.evaluate(t_imgs, t_poses, dirs)
    white = sum(float(-10 * torch.log10(((1 - im) ** 2).mean())) for im in t_imgs) / len(t_imgs)
    print("\nTRAIN", [(h["step"], round(h["psnr"], 2), round(h["loss"], 5), round(h["rm_s"], 1), h["lr"])
                      for h in hist], "\nTEST psnr", round(psnr, 2), [round(v, 2) for v in per_view],
          "white-image baseline", round(white, 2))
    assert psnr > white + 8.0 and psnr > 25.0
    assert abs(hist[-1]["lr"] - hp.lr * 0.01) < 1e-9 and hist[-1]["skipped"] == 0
    # checkpoint round trip (reference key layout) into a fresh trainer and into the NGP mirror
    path = str(tmp_path / "ck.ckpt")
    tr.save(path)
    tr2 = Trainer(hp, ds, device=gpu)
    tr2.load(path)
    assert torch.equal(tr2.step.p16[:tr.step.n_params], tr.step.p16[:tr.step.n_params])
    assert torch.equal(tr2.step.bitfield, tr.step.bitfield)
    psnr2, _ = tr2.evaluate(t_imgs, t_poses, dirs)
    assert abs(psnr2 - psnr) < 1e-3
    sd = torch.load(path, map_location="cpu", weights_only=True)["state_dict"]
    from mfnerf.networks import NGP
    m = NGP(0.5, hp)
    m.load_state_dict({k[6:]: v for k, v in sd.items() if k.startswith("model.")}, strict=False)
    assert torch.equal(m.rgb_net.params.detach(), tr.step.params[tr.step.off_rgb:tr.step.off_table].cpu())


def test_trainer_mixedfeature_rgb128_learns_a_scene(gpu):
    """The MF benchmark configuration's field (benchmark_synthetic_mf.sh: --grid MixedFeature
    --N_tables 8 --rgb_channels 128) through the whole fused step: shared-table fixed-point table
    gradient, width-128 MFMA head, pipelined graphs."""
    imgs, poses, dirs, K = _ball_views(100)
    t_imgs, t_poses, _, _ = _ball_views(4, seed=7)
    ds = data.DeviceDataset(imgs, poses, dirs, K=K, img_wh=(64, 64), device=gpu, seed=5)
    hp = HParams(batch_size=4096, T=16, num_epochs=1, steps_per_epoch=800, grid="MixedFeature", N_tables=8,
                 rgb_channels=128, lr=2e-2)
    tr = Trainer(hp, ds, device=gpu)
    hist = tr.fit(log_every=400)
    psnr, _ = tr.evaluate(t_imgs, t_poses, dirs)
    white = sum(float(-10 * torch.log10(((1 - im) ** 2).mean())) for im in t_imgs) / len(t_imgs)
    print("\nMF128 TRAIN", [(h["step"], round(h["psnr"], 2)) for h in hist], "TEST psnr", round(psnr, 2),
          "white", round(white, 2))
    assert psnr > white + 6.0 and hist[-1]["skipped"] == 0


def test_trainer_on_a_colmap_scene(gpu):
    """The real-scene configuration (benchmark_mipnerf360_mf.sh: colmap, --scale 16): 6 cascades,
    exp_step_factor 1/256 marching, black background, the occupancy erode -- on the generated COLMAP
    scene of tests/golden (noise images: the check is that every piece runs and stays finite)."""
    import os
    from conftest import ROOT
    ds0 = data.ColmapDataset(os.path.join(ROOT, "tests", "golden", "colmap_scene"), split="train")
    ds = data.DeviceDataset.from_dataset(ds0, device=gpu, seed=2)
    hp = HParams(dataset_name="colmap", scale=16.0, batch_size=1024, T=16, num_epochs=1, steps_per_epoch=300,
                 grid="MixedFeature", N_tables=8, rgb_channels=128)
    tr = Trainer(hp, ds, device=gpu)
    assert tr.step.cascades == 6
    hist = tr.fit(log_every=100)
    assert all(math.isfinite(h["loss"]) for h in hist) and hist[-1]["skipped"] == 0
    assert torch.isfinite(tr.step.params).all()


def test_sample_rays_prep_matches_aabb_and_clamp(gpu):
    """The fused draw + march prologue: the drawn rays equal mfnerf_sample_rays' (same counter), and
    hits_t equals ray_aabb_intersect + the near clamp (rendering.py:27-29) on them, bit for bit; the
    noise is U[0,1) and fresh on every draw."""
    from mfnerf import vren
    g = torch.Generator().manual_seed(1)
    n_img, hw, N = 4, 500, 4096
    imgs = torch.rand(n_img, hw, 3, generator=g)
    poses = torch.cat([torch.linalg.qr(torch.randn(n_img, 3, 3, generator=g))[0],
                       torch.rand(n_img, 3, 1, generator=g) * 3 - 1.5], 2)
    dirs = torch.randn(hw, 3, generator=g)
    center, half = torch.zeros(1, 3, device=gpu), torch.full((1, 3), 0.5, device=gpu)
    a = data.DeviceDataset(imgs, poses, dirs, device=gpu, seed=4)
    b = data.DeviceDataset(imgs, poses, dirs, device=gpu, seed=4)
    out_a, out_b = torch.empty(3, N, 3, device=gpu), torch.empty(3, N, 3, device=gpu)
    hits, noise = torch.empty(N, 2, device=gpu), torch.empty(N, device=gpu)
    a.sample(out_a)
    b.sample(out_b, prep=(center, half, 0.01, hits, noise))
    assert torch.equal(out_a, out_b)
    _, ht, _ = vren.ray_aabb_intersect(out_b[0].contiguous(), out_b[1].contiguous(), center, half, 1)
    t1 = ht[:, 0, 0]
    t1[(t1 >= 0) & (t1 < 0.01)] = 0.01
    assert torch.equal(hits, ht[:, 0])
    assert (hits[:, 0] >= 0).sum() > 100 and (hits[:, 0] < 0).sum() > 100
    assert float(noise.min()) >= 0.0 and float(noise.max()) < 1.0 and abs(float(noise.mean()) - 0.5) < 0.02
    n1 = noise.clone()
    b.sample(out_b, prep=(center, half, 0.01, hits, noise))
    assert not torch.equal(n1, noise)

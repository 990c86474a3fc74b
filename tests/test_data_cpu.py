"""Host-side data and training-harness logic: NSVF loader (datasets/nsvf.py) on a generated mini
scene, ray utilities (datasets/ray_utils.py), the LR schedule (train.py:136-142)."""
import math
import os

import numpy as np
import pytest
import torch

from mfnerf import data
from mfnerf.trainer import HParams, cosine_lr


def _write_scene(root, n=3, W=800, alpha=True):
    from PIL import Image
    os.makedirs(os.path.join(root, "rgb"))
    os.makedirs(os.path.join(root, "pose"))
    with open(os.path.join(root, "intrinsics.txt"), "w") as f:
        f.write("1111.111 0. 0. 0.\n0. 0. 0. 0.\n0. 0. 0. 0.\n0. 0. 0. 0.\n")
    np.savetxt(os.path.join(root, "bbox.txt"), np.array([[-0.6, -1.2, -0.3, 0.8, 1.0, 0.9, 0.01]]))
    g = np.random.default_rng(0)
    imgs, poses = [], []
    for split in (0, 2):
        for i in range(n):
            rgba = g.integers(0, 256, (W, W, 4), dtype=np.uint8)
            Image.fromarray(rgba if alpha else rgba[..., :3]).save(os.path.join(root, "rgb", f"{split}_{i:04d}.png"))
            c2w = np.eye(4)
            c2w[:3, 3] = g.uniform(-3, 3, 3)
            np.savetxt(os.path.join(root, "pose", f"{split}_{i:04d}.txt"), c2w)
            if split == 0:
                imgs.append(rgba)
                poses.append(c2w)
    return imgs, poses


def test_nsvf_loader_matches_reference_semantics(tmp_path):
    root = str(tmp_path / "Synthetic_NeRF" / "Lego")
    imgs, poses = _write_scene(root)
    ds = data.NSVFDataset(root, split="train")
    assert ds.img_wh == (800, 800) and ds.rays.shape == (3, 800 * 800, 3) and ds.poses.shape == (3, 3, 4)
    # bbox: shift = centre, scale = max half extent * 1.05 * 1.1 (Lego fix)
    lo, hi = np.array([-0.6, -1.2, -0.3]), np.array([0.8, 1.0, 0.9])
    shift, scale = (lo + hi) / 2, (hi - lo).max() / 2 * 1.05 * 1.1
    assert np.allclose(ds.shift, shift) and math.isclose(ds.scale, scale)
    assert torch.allclose(ds.poses[1, :, 3], torch.tensor((poses[1][:3, 3] - shift) / (2 * scale), dtype=torch.float32))
    # alpha blended onto white (color_utils.py:22-25)
    a = imgs[2].astype(np.float32) / 255
    ref = a[..., :3] * a[..., 3:] + (1 - a[..., 3:])
    assert np.allclose(ds.rays[2].numpy(), ref.reshape(-1, 3), atol=1e-6)
    assert torch.allclose(ds.K, torch.tensor([[1111.111, 0, 400], [0, 1111.111, 400], [0, 0, 1]]))
    test = data.NSVFDataset(root, split="test")
    assert test.rays.shape[0] == 3  # Synthetic test split = prefix 2_


def test_ray_directions_and_rays():
    K = torch.tensor([[100.0, 0, 32], [0, 90.0, 24], [0, 0, 1]])
    d = data.get_ray_directions(48, 64, K)
    assert d.shape == (48 * 64, 3)
    r, c = 7, 13  # row-major (h, w): u = column, v = row, through the pixel centre
    assert torch.allclose(d[r * 64 + c], torch.tensor([(c - 32 + 0.5) / 100, (r - 24 + 0.5) / 90, 1.0]))
    c2w = torch.randn(5, 3, 4)
    o, dd = data.get_rays(d[:5], c2w)
    for i in range(5):
        assert torch.allclose(dd[i], c2w[i, :, :3] @ d[i], atol=1e-6) and torch.equal(o[i], c2w[i, :, 3])


def test_cosine_lr_matches_torch_scheduler():
    hp = HParams(num_epochs=30, lr=1e-2)
    opt = torch.optim.SGD([torch.zeros(1, requires_grad=True)], lr=hp.lr)
    sch = torch.optim.lr_scheduler.CosineAnnealingLR(opt, hp.num_epochs - 1, hp.lr * 0.01)
    for e in range(hp.num_epochs):
        assert math.isclose(cosine_lr(e, hp), opt.param_groups[0]["lr"], rel_tol=1e-9), e
        opt.step()
        sch.step()
    assert math.isclose(cosine_lr(29, hp), 1e-4, rel_tol=1e-9)


def test_ball_scene_renders_hits_and_background():
    sc = data.BallScene(n_balls=1, seed=0)
    sc.c[:] = 0.0
    sc.r[:] = 0.25
    o = torch.tensor([[0.0, 0.0, -2.0], [0.0, 1.0, -2.0]])
    d = torch.tensor([[0.0, 0.0, 1.0], [0.0, 0.0, 1.0]])
    out = sc.render(o, d)
    assert torch.allclose(out[0], sc.rgb[0]) and torch.equal(out[1], torch.ones(3))

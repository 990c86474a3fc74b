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
    # textured: the hit point (0, 0, -0.25) has sin(f*0) = 0, so the pattern vanishes there;
    # an off-axis hit carries it, the background stays white
    sc.texture_freq = 40.0
    o2 = torch.tensor([[0.0, 0.0, -2.0], [0.1, 0.07, -2.0], [0.0, 1.0, -2.0]])
    d2 = torch.tensor([[0.0, 0.0, 1.0]] * 3)
    out2 = sc.render(o2, d2)
    assert torch.allclose(out2[0], sc.rgb[0]) and torch.equal(out2[2], torch.ones(3))
    z = -math.sqrt(0.25 ** 2 - 0.1 ** 2 - 0.07 ** 2)
    pat = math.sin(4.0) * math.sin(2.8) * math.sin(40.0 * z)
    want = (sc.rgb[0].double() + 0.3 * pat * torch.tensor([1.0, -0.6, 0.8], dtype=torch.float64)).clamp(0, 1)
    assert torch.allclose(out2[1].double(), want, atol=1e-6)


GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_colmap_loader_matches_reference_golden():
    """ColmapDataset vs the reference's datasets/colmap.py run on the same generated sparse model
    (tests/golden/make_golden_colmap.py): K, img_wh, centred + scaled poses of both splits (name
    order, every-8th test image), the centred point cloud and the pixel values."""
    z = np.load(os.path.join(GOLD, "golden_colmap.npz"))
    root = os.path.join(GOLD, "colmap_scene")
    for split in ("train", "test"):
        ds = data.ColmapDataset(root, split=split)
        assert ds.poses.shape == z[f"{split}_poses"].shape
        assert np.allclose(ds.poses.numpy(), z[f"{split}_poses"], atol=1e-6, rtol=0)
        assert np.array_equal(ds.rays.numpy(), z[f"{split}_rays"])
    assert np.array_equal(ds.K.numpy(), z["K"]) and tuple(ds.img_wh) == tuple(z["img_wh"])
    assert np.allclose(ds.pts3d, z["pts3d"], atol=1e-9)
    # the nearest camera sits at distance 1 after the scaling
    allp = data.ColmapDataset(root, split="val", read_images=False).poses
    assert abs(float(allp[..., 3].norm(dim=-1).min()) - 1.0) < 1e-6


def test_colmap_readers_and_360_folder(tmp_path):
    """Binary readers on a hand-built model (SIMPLE_RADIAL intrinsics, an image with 2D points) and
    the mip-NeRF 360 images_{1/downsample} folder rule (colmap.py:53-56)."""
    import struct
    from PIL import Image
    root = tmp_path / "360_v2" / "garden"
    (root / "sparse" / "0").mkdir(parents=True)
    (root / "images_4").mkdir()
    with open(root / "sparse/0/cameras.bin", "wb") as f:
        f.write(struct.pack("<Q", 1) + struct.pack("<iiQQ", 1, 2, 80, 40) + struct.pack("<4d", 50.0, 40.0, 20.0, 0.1))
    q = np.array([0.9, 0.1, -0.3, 0.2])
    q /= np.linalg.norm(q)
    with open(root / "sparse/0/images.bin", "wb") as f:
        f.write(struct.pack("<Q", 2))
        for k, name in enumerate(["b.jpg", "a.jpg"]):
            f.write(struct.pack("<i4d3di", 7 + k, *q, 1.0 + k, 2.0, -1.0, 1) + name.encode() + b"\0")
            f.write(struct.pack("<Q", 2) + struct.pack("<ddq", 1.0, 2.0, 5) * 2)
    with open(root / "sparse/0/points3D.bin", "wb") as f:
        f.write(struct.pack("<Q", 2))
        for p in range(2):
            f.write(struct.pack("<Q3d3Bd", p, 0.5 * p, -1.0, 2.0, 1, 2, 3, 0.5) + struct.pack("<Q", 1)
                    + struct.pack("<ii", 7, 0))
    for name in ("a.jpg", "b.jpg"):
        Image.fromarray(np.zeros((10, 20, 3), np.uint8)).save(root / "images_4" / name)
    cams = data.read_colmap_cameras(str(root / "sparse/0/cameras.bin"))
    assert cams[1][0] == "SIMPLE_RADIAL" and cams[1][1:3] == (80, 40)
    ims = data.read_colmap_images(str(root / "sparse/0/images.bin"))
    assert [v[0] for v in ims.values()] == ["b.jpg", "a.jpg"] and np.allclose(ims[8][2], [2.0, 2.0, -1.0])
    R = data.qvec_to_rotmat(q)
    assert np.allclose(R @ R.T, np.eye(3), atol=1e-12) and abs(np.linalg.det(R) - 1) < 1e-12
    assert np.allclose(data.read_colmap_points3d(str(root / "sparse/0/points3D.bin")), [[0, -1, 2], [0.5, -1, 2]])
    ds = data.ColmapDataset(str(root), split="val", downsample=0.25)
    assert ds.img_wh == (20, 10) and ds.img_paths[0].endswith(os.path.join("images_4", "a.jpg"))
    assert torch.allclose(ds.K, torch.tensor([[12.5, 0, 10.0], [0, 12.5, 5.0], [0, 0, 1]]))
    assert ds.rays.shape == (2, 200, 3)

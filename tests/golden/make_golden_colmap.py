"""Golden vectors for the COLMAP loader (mfnerf.data.ColmapDataset), made by running the REFERENCE's
datasets/colmap.py (ColmapDataset with its colmap_utils readers and ray_utils.center_poses) on a
small generated scene.

The scene (tests/golden/colmap_scene/: sparse/0/{cameras,images,points3D}.bin in COLMAP's binary
layout + 12 small PNGs) is written by this script from a fixed seed; the images are stored under
names out of file order, so the name sort and the every-8th test split are exercised, and images
and points carry 2D-point / track lists the readers must skip.  The reference's third-party imports
that are absent here are stubbed with the behaviour its loader relies on: imageio.imread (PIL),
cv2.resize (identity at the native size, the only size this scene is read at) and
kornia.create_meshgrid (the pixel grid; directions are not part of the fixture).  Only data is
written: golden_colmap.npz.

Run: python tests/golden/make_golden_colmap.py   (needs /root/reference; CPU only)
"""
import os
import struct
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("MFNERF_REFERENCE", "/root/reference")
SCENE = os.path.join(HERE, "colmap_scene")
sys.dont_write_bytecode = True

W, H, N_IMG, N_PTS = 24, 18, 12, 40


def write_scene(root, seed=0):
    from PIL import Image
    g = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, "sparse", "0"), exist_ok=True)
    os.makedirs(os.path.join(root, "images"), exist_ok=True)
    with open(os.path.join(root, "sparse/0/cameras.bin"), "wb") as f:  # camera 1: PINHOLE
        f.write(struct.pack("<Q", 1))
        f.write(struct.pack("<iiQQ", 1, 1, W, H))
        f.write(struct.pack("<4d", 21.5, 22.25, 11.75, 8.5))
    names = [f"frame_{i:03d}.png" for i in range(N_IMG)]
    order = g.permutation(N_IMG)
    with open(os.path.join(root, "sparse/0/images.bin"), "wb") as f:
        f.write(struct.pack("<Q", N_IMG))
        for k, i in enumerate(order):
            q = g.normal(size=4)
            q /= np.linalg.norm(q)
            t = g.uniform(-2, 2, 3)
            f.write(struct.pack("<i4d3di", 100 + k, *q, *t, 1))
            f.write(names[i].encode() + b"\0")
            n2 = int(g.integers(0, 4))
            f.write(struct.pack("<Q", n2))
            for _ in range(n2):
                f.write(struct.pack("<ddq", *g.uniform(0, W, 2), int(g.integers(-1, N_PTS))))
    with open(os.path.join(root, "sparse/0/points3D.bin"), "wb") as f:
        f.write(struct.pack("<Q", N_PTS))
        for p in range(N_PTS):
            f.write(struct.pack("<Q3d3Bd", p + 1, *g.normal(0, 1.5, 3), *[int(c) for c in g.integers(0, 256, 3)],
                                float(g.uniform())))
            tl = int(g.integers(0, 3))
            f.write(struct.pack("<Q", tl))
            for _ in range(tl):
                f.write(struct.pack("<ii", int(g.integers(1, N_IMG)), int(g.integers(0, 5))))
    for i in range(N_IMG):
        Image.fromarray(g.integers(0, 256, (H, W, 3), dtype=np.uint8)).save(os.path.join(root, "images", names[i]))


def install_stubs():
    import torch
    from PIL import Image
    im = types.ModuleType("imageio")
    im.imread = lambda p: np.asarray(Image.open(p))
    sys.modules["imageio"] = im
    cv = types.ModuleType("cv2")

    def resize(img, wh):
        if (img.shape[1], img.shape[0]) != tuple(wh):
            raise NotImplementedError("the golden scene is read at its native size")
        return img

    cv.resize = resize
    sys.modules["cv2"] = cv
    ko = types.ModuleType("kornia")

    def create_meshgrid(h, w, normalized=True, device="cpu"):
        ys, xs = torch.meshgrid(torch.arange(h, dtype=torch.float32), torch.arange(w, dtype=torch.float32),
                                indexing="ij")
        return torch.stack([xs, ys], -1)[None]

    ko.create_meshgrid = create_meshgrid
    sys.modules["kornia"] = ko
    sys.path.insert(0, REF)


def main():
    write_scene(SCENE)
    install_stubs()
    import warnings
    warnings.filterwarnings("ignore")
    from datasets.colmap import ColmapDataset
    out = {}
    for split in ("train", "test"):
        ds = ColmapDataset(SCENE, split=split)
        out[f"{split}_poses"] = ds.poses.numpy()
        out[f"{split}_rays"] = ds.rays.numpy()
    out["K"] = ds.K.numpy()
    out["img_wh"] = np.array(ds.img_wh)
    out["pts3d"] = np.asarray(ds.pts3d)
    np.savez_compressed(os.path.join(HERE, "golden_colmap.npz"), **out)
    print("wrote golden_colmap.npz:", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()

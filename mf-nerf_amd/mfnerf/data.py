"""Training data for the step: the reference's NSVF dataset (datasets/nsvf.py:12-100), its ray
utilities (datasets/ray_utils.py:8-70) and image reader (datasets/color_utils.py:19-31), and a
GPU-resident dataset whose per-step batch (random image + pixel per ray -> rays_o, rays_d, rgb;
datasets/base.py:22-35 + train.py:93-105) is one HIP launch (mfnerf_sample_rays), so the data side
of a training step stays on the device and inside the step's graph.

Also an analytic scene (opaque coloured balls in the unit box, exact ray-sphere first hits, white
background) that renders ground-truth views of any camera: the image has no datasets, so tests and
bench.py train on it.
"""
import glob
import math
import os
import struct

import numpy as np
import torch

from ._lib import call, ptr, stream


# ---------------------------------------------------------------------------- ray utilities
def get_ray_directions(H, W, K, device="cpu", random=False, flatten=True):
    """ray_utils.py:8-47: camera-frame directions [right down front] through pixel centres
    (kornia create_meshgrid(H, W, normalized=False): u = column, v = row)."""
    v, u = torch.meshgrid(torch.arange(H, dtype=torch.float32, device=device),
                          torch.arange(W, dtype=torch.float32, device=device), indexing="ij")
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    if random:
        d = torch.stack([(u - cx + torch.rand_like(u)) / fx, (v - cy + torch.rand_like(v)) / fy, torch.ones_like(u)], -1)
    else:
        d = torch.stack([(u - cx + 0.5) / fx, (v - cy + 0.5) / fy, torch.ones_like(u)], -1)
    return d.reshape(-1, 3) if flatten else d


def get_rays(directions, c2w):
    """ray_utils.py:50-70: world-frame (rays_o, rays_d) for (N,3) directions and (3,4) / (N,3,4) poses."""
    if c2w.ndim == 2:
        rays_d = directions @ c2w[:, :3].T
    else:
        rays_d = (directions[:, None, :] @ c2w[..., :3].transpose(1, 2))[:, 0]
    rays_o = c2w[..., 3].expand_as(rays_d)
    return rays_o, rays_d


def read_image(path, img_wh, blend_a=True):
    """color_utils.py:19-31: float RGB in [0,1], alpha blended onto white, flattened (h*w, 3).
    The reference resizes with cv2 (INTER_LINEAR); cv2 is not in this image, so a size change uses
    PIL's bilinear filter instead (identical at downsample 1.0, where no resize happens)."""
    from PIL import Image
    im = Image.open(path)
    img = np.asarray(im).astype(np.float32) / 255.0
    if img.ndim == 2:
        img = np.repeat(img[..., None], 3, -1)
    if img.shape[2] == 4:
        img = img[..., :3] * img[..., -1:] + (1 - img[..., -1:]) if blend_a else img[..., :3] * img[..., -1:]
    if (img.shape[1], img.shape[0]) != tuple(img_wh):
        chans = [np.asarray(Image.fromarray(img[..., c]).resize(tuple(img_wh), Image.BILINEAR)) for c in range(3)]
        img = np.stack(chans, -1)
    return img.reshape(-1, 3)


# ---------------------------------------------------------------------------- NSVF
class NSVFDataset:
    """datasets/nsvf.py: intrinsics.txt / bbox.txt / pose/*.txt / rgb/*.png under root_dir.
    Poses are shifted by the bbox centre and scaled by 2*scale (scene inside [-0.5,0.5]^3, with the
    reference's 1.05 enlargement and its Lego (1.1) / Mic (1.2) fixes); splits by file prefix
    (train 0_, val 1_, test 2_ for Synthetic scenes, 1_ for real ones)."""

    def __init__(self, root_dir, split="train", downsample=1.0):
        self.root_dir, self.split, self.downsample = root_dir, split, downsample
        self.read_intrinsics()
        xyz_min, xyz_max = np.loadtxt(os.path.join(root_dir, "bbox.txt"))[:6].reshape(2, 3)
        self.shift = (xyz_max + xyz_min) / 2
        self.scale = (xyz_max - xyz_min).max() / 2 * 1.05
        if "Mic" in root_dir:
            self.scale *= 1.2
        elif "Lego" in root_dir:
            self.scale *= 1.1
        self.read_meta(split)

    def read_intrinsics(self):
        r = self.root_dir
        if "Synthetic" in r or "Ignatius" in r:
            with open(os.path.join(r, "intrinsics.txt")) as f:
                fx = fy = float(f.readline().split()[0]) * self.downsample
            if "Synthetic" in r:
                w = h = int(800 * self.downsample)
            else:
                w, h = int(1920 * self.downsample), int(1080 * self.downsample)
            K = np.float32([[fx, 0, w / 2], [0, fy, h / 2], [0, 0, 1]])
        else:
            K = np.loadtxt(os.path.join(r, "intrinsics.txt"), dtype=np.float32)[:3, :3]
            if "BlendedMVS" in r:
                w, h = int(768 * self.downsample), int(576 * self.downsample)
            elif "Tanks" in r:
                w, h = int(1920 * self.downsample), int(1080 * self.downsample)
            else:
                raise ValueError(f"unknown NSVF scene family: {r}")
            K[:2] *= self.downsample
        self.K = torch.FloatTensor(K)
        self.directions = get_ray_directions(h, w, self.K)
        self.img_wh = (w, h)

    def read_meta(self, split):
        r = self.root_dir
        prefix = {"train": "0_", "trainval": "[0-1]_", "trainvaltest": "[0-2]_", "val": "1_"}.get(split)
        if prefix is None:
            if split != "test":
                raise ValueError(f"{split} split not recognized!")
            prefix = "2_" if "Synthetic" in r else "1_"
        img_paths = sorted(glob.glob(os.path.join(r, "rgb", prefix + "*.png")))
        pose_paths = sorted(glob.glob(os.path.join(r, "pose", prefix + "*.txt")))
        poses, rays = [], []
        for ip, pp in zip(img_paths, pose_paths):
            c2w = np.loadtxt(pp)[:3]
            c2w[:, 3] -= self.shift
            c2w[:, 3] /= 2 * self.scale
            poses.append(c2w)
            img = read_image(ip, self.img_wh)
            if "Jade" in r or "Fountain" in r:
                img[np.all(img <= 0.1, axis=-1)] = 1.0
            rays.append(img)
        self.rays = torch.FloatTensor(np.stack(rays)) if rays else torch.zeros(0, 0, 3)
        self.poses = torch.FloatTensor(np.stack(poses)) if poses else torch.zeros(0, 3, 4)


# ---------------------------------------------------------------------------- COLMAP
# The sparse-model readers the reference's ColmapDataset uses (datasets/colmap_utils.py:108-260, after
# COLMAP's own binary writers): little-endian; only the fields the dataset reads are kept.
_COLMAP_MODELS = {0: ("SIMPLE_PINHOLE", 3), 1: ("PINHOLE", 4), 2: ("SIMPLE_RADIAL", 4), 3: ("RADIAL", 5),
                  4: ("OPENCV", 8), 5: ("OPENCV_FISHEYE", 8), 6: ("FULL_OPENCV", 12), 7: ("FOV", 5),
                  8: ("SIMPLE_RADIAL_FISHEYE", 4), 9: ("RADIAL_FISHEYE", 5), 10: ("THIN_PRISM_FISHEYE", 12)}


def _read(path):
    with open(path, "rb") as f:
        return f.read()


def read_colmap_cameras(path):
    """cameras.bin -> {camera_id: (model name, width, height, params f64)}.  Layout: u64 count; per
    camera i32 id, i32 model id, u64 width, u64 height, f64 params[n(model)]."""
    buf = _read(path)
    (n,) = struct.unpack_from("<Q", buf, 0)
    off, cams = 8, {}
    for _ in range(n):
        cid, mid, w, h = struct.unpack_from("<iiQQ", buf, off)
        name, k = _COLMAP_MODELS[mid]
        cams[cid] = (name, w, h, np.array(struct.unpack_from(f"<{k}d", buf, off + 24)))
        off += 24 + 8 * k
    return cams


def read_colmap_images(path):
    """images.bin -> {image_id: (name, qvec (w, x, y, z), tvec)} in file order.  Layout: u64 count;
    per image i32 id, f64 qvec[4], f64 tvec[3], i32 camera id, NUL-terminated name, u64 n_points2D,
    n x (f64 x, f64 y, i64 point3D id)."""
    buf = _read(path)
    (n,) = struct.unpack_from("<Q", buf, 0)
    off, ims = 8, {}
    for _ in range(n):
        (iid,) = struct.unpack_from("<i", buf, off)
        q = np.array(struct.unpack_from("<4d", buf, off + 4))
        t = np.array(struct.unpack_from("<3d", buf, off + 36))
        end = buf.index(b"\0", off + 64)
        (n2d,) = struct.unpack_from("<Q", buf, end + 1)
        ims[iid] = (buf[off + 64:end].decode("utf-8"), q, t)
        off = end + 9 + 24 * n2d
    return ims


def read_colmap_points3d(path):
    """points3D.bin -> (N, 3) f64 xyz in file order.  Layout: u64 count; per point u64 id, f64 xyz[3],
    u8 rgb[3], f64 error, u64 track length, track x (i32 image id, i32 point2D index)."""
    buf = _read(path)
    (n,) = struct.unpack_from("<Q", buf, 0)
    off, xyz = 8, np.empty((n, 3))
    for i in range(n):
        xyz[i] = struct.unpack_from("<3d", buf, off + 8)
        (tl,) = struct.unpack_from("<Q", buf, off + 43)
        off += 51 + 8 * tl
    return xyz


def qvec_to_rotmat(q):
    """COLMAP quaternion (w, x, y, z) -> rotation matrix, in colmap_utils.py:272-282's term order."""
    w, x, y, z = q
    return np.array([
        [1 - 2 * y ** 2 - 2 * z ** 2, 2 * x * y - 2 * w * z, 2 * z * x + 2 * w * y],
        [2 * x * y + 2 * w * z, 1 - 2 * x ** 2 - 2 * z ** 2, 2 * y * z - 2 * w * x],
        [2 * z * x - 2 * w * y, 2 * y * z + 2 * w * x, 1 - 2 * x ** 2 - 2 * y ** 2]])


def _normalize(v):
    return v / np.linalg.norm(v)


def average_pose(poses, pts3d=None):
    """ray_utils.py:108-147: centre = mean of the point cloud (else of the camera centres), z = the
    normalised mean z axis, x = normalize(mean y axis x z), y = z x x."""
    center = pts3d.mean(0) if pts3d is not None else poses[..., 3].mean(0)
    z = _normalize(poses[..., 2].mean(0))
    y_ = poses[..., 1].mean(0)
    x = _normalize(np.cross(y_, z))
    y = np.cross(z, x)
    return np.stack([x, y, z, center], 1)


def center_poses(poses, pts3d=None):
    """ray_utils.py:150-178: poses (and points) expressed in the frame of the average pose."""
    avg = np.eye(4)
    avg[:3] = average_pose(poses, pts3d)
    inv = np.linalg.inv(avg)
    homo = np.concatenate([poses, np.tile(np.array([0, 0, 0, 1]), (len(poses), 1, 1))], 1)
    out = (inv @ homo)[:, :3]
    if pts3d is None:
        return out
    return out, pts3d @ inv[:, :3].T + inv[:, 3:].T


class ColmapDataset:
    """datasets/colmap.py:15-159 for COLMAP scenes (the mip-NeRF 360 configs, e.g. garden): camera 1's
    intrinsics scaled by `downsample` (SIMPLE_RADIAL / PINHOLE / OPENCV; distortion ignored, as
    there), cam2world poses in image-name order centred on the sparse point cloud and scaled so the
    nearest camera is at distance 1, every 8th image of that order as the test split, images read
    without alpha blending; 360_v2 scenes at downsample < 1 read images_{1/downsample}.  The HDR-NeRF
    branches and the 'test_traj' spiral are out of scope."""

    def __init__(self, root_dir, split="train", downsample=1.0, read_images=True):
        self.root_dir, self.split, self.downsample = root_dir, split, downsample
        self.read_intrinsics()
        self.read_meta(split, read_images)

    def read_intrinsics(self):
        model, W, H, p = read_colmap_cameras(os.path.join(self.root_dir, "sparse/0/cameras.bin"))[1]
        ds = self.downsample
        h, w = int(H * ds), int(W * ds)
        self.img_wh = (w, h)
        if model == "SIMPLE_RADIAL":
            fx = fy = p[0] * ds
            cx, cy = p[1] * ds, p[2] * ds
        elif model in ("PINHOLE", "OPENCV"):
            fx, fy, cx, cy = p[0] * ds, p[1] * ds, p[2] * ds, p[3] * ds
        else:
            raise ValueError(f"Please parse the intrinsics for camera model {model}!")
        self.K = torch.FloatTensor([[fx, 0, cx], [0, fy, cy], [0, 0, 1]])
        self.directions = get_ray_directions(h, w, self.K)

    def read_meta(self, split, read_images=True):
        r = self.root_dir
        if split == "test_traj" or "HDR-NeRF" in r:
            raise NotImplementedError("COLMAP test_traj / HDR-NeRF splits are out of scope")
        ims = read_colmap_images(os.path.join(r, "sparse/0/images.bin"))
        names = [v[0] for v in ims.values()]
        perm = np.argsort(names)
        folder = f"images_{int(1 / self.downsample)}" if "360_v2" in r and self.downsample < 1 else "images"
        paths = [os.path.join(r, folder, nm) for nm in sorted(names)]
        w2c = np.stack([np.concatenate([np.concatenate([qvec_to_rotmat(q), t.reshape(3, 1)], 1),
                                        np.array([[0, 0, 0, 1.0]])], 0) for _, q, t in ims.values()])
        poses = np.linalg.inv(w2c)[perm, :3]
        pts = read_colmap_points3d(os.path.join(r, "sparse/0/points3D.bin"))
        self.poses, self.pts3d = center_poses(poses, pts)
        scale = np.linalg.norm(self.poses[..., 3], axis=-1).min()
        self.poses[..., 3] /= scale
        self.pts3d /= scale
        keep = list(range(len(paths)))
        if split == "train":
            keep = [i for i in keep if i % 8 != 0]
        elif split == "test":
            keep = [i for i in keep if i % 8 == 0]
        self.img_paths = [paths[i] for i in keep]
        poses = self.poses[keep]
        if read_images:
            rays = [read_image(pth, self.img_wh, blend_a=False) for pth in self.img_paths]
            self.rays = torch.FloatTensor(np.stack(rays)) if rays else torch.zeros(0, 0, 3)
        self.poses = torch.FloatTensor(poses)


# ---------------------------------------------------------------------------- GPU-resident batches
class DeviceDataset:
    """Images (n_img, hw, 3), poses (n_img, 3, 4) and camera directions (hw, 3) resident in HBM;
    sample(out) draws one training batch into a (3, N, 3) buffer with one launch (graph-safe: the
    draw counter lives on the device).  strategy: 'all_images' or 'same_image' (base.py:25-28)."""

    def __init__(self, images, poses, directions, K=None, img_wh=None, device="cuda", seed=0,
                 strategy="all_images"):
        self.images = images.float().contiguous().to(device)
        self.poses = poses.float().contiguous().to(device)
        self.directions = directions.float().contiguous().to(device)
        self.K, self.img_wh = K, img_wh
        self.n_img, self.hw = self.images.shape[0], self.images.shape[1]
        assert self.poses.shape == (self.n_img, 3, 4) and self.directions.shape == (self.hw, 3)
        self.seed = int(seed)
        self.same_image = {"all_images": 0, "same_image": 1}[strategy]
        self.calls = torch.zeros(2, dtype=torch.int64, device=device)  # device draw counter + its launch ticket

    @classmethod
    def from_dataset(cls, ds, device="cuda", **kw):
        """From an NSVFDataset or a ColmapDataset (rays, poses, directions, K, img_wh)."""
        return cls(ds.rays, ds.poses, ds.directions, K=ds.K, img_wh=ds.img_wh, device=device, **kw)

    from_nsvf = from_dataset

    def sample(self, out, img_idx=None, pix_idx=None, prep=None):
        """out (3, N, 3) f32 <- [rays_o | rays_d | rgb] of N random rays.  prep = (center, half_size,
        near, hits_t (N,2), noise (N)): also the march prologue (AABB hit, near clamp, noise) of the
        drawn rays, in the same launch (mfnerf_sample_rays_prep)."""
        n = out.shape[1]
        if prep is not None:
            center, half_size, near, hits_t, noise = prep
            call("mfnerf_sample_rays_prep", ptr(self.images), ptr(self.poses), ptr(self.directions), self.n_img,
                 self.hw, n, self.same_image, self.seed, ptr(self.calls), ptr(out), ptr(center), ptr(half_size),
                 float(near), ptr(hits_t), ptr(noise), stream())
            return out
        call("mfnerf_sample_rays", ptr(self.images), ptr(self.poses), ptr(self.directions), self.n_img, self.hw, n,
             self.same_image, self.seed, ptr(self.calls), ptr(out), ptr(img_idx), ptr(pix_idx), stream())
        return out


# ---------------------------------------------------------------------------- analytic scene
class BallScene:
    """Opaque coloured balls inside [-0.5, 0.5]^3; render(o, d) = colour of the first ball hit,
    white where nothing is hit (the synthetic-scene background of rendering.py:153-155).  With
    texture_freq > 0 each ball's colour carries a world-space sin(f x) sin(f y) sin(f z) pattern."""

    def __init__(self, n_balls=8, seed=0, radius=(0.08, 0.2)):
        g = torch.Generator().manual_seed(seed)
        self.r = torch.rand(n_balls, generator=g) * (radius[1] - radius[0]) + radius[0]
        self.c = (torch.rand(n_balls, 3, generator=g) - 0.5) * (1.0 - 2 * self.r[:, None]).clamp(min=0)
        self.rgb = torch.rand(n_balls, 3, generator=g) * 0.8 + 0.1
        self.texture_freq = 0.0

    @classmethod
    def matching_grid(cls, seed=0, n_balls=12, radius=(0.065, 0.18)):
        """The balls of synthetic.ball_density_grid(seed=seed) (the bench's calibrated occupancy)."""
        sc = cls(n_balls=n_balls, seed=seed, radius=radius)
        g = np.random.default_rng(seed)
        sc.c = torch.from_numpy(g.uniform(-0.5 + radius[1], 0.5 - radius[1], size=(n_balls, 3))).float()
        sc.r = torch.from_numpy(g.uniform(radius[0], radius[1], size=n_balls)).float()
        return sc

    def render(self, o, d):
        o, d = o.double(), d.double()
        c, r, rgb = (t.double().to(o.device) for t in (self.c, self.r, self.rgb))
        dn = d / d.norm(dim=-1, keepdim=True)
        oc = o[:, None, :] - c[None]                                   # (N, B, 3)
        b = (oc * dn[:, None, :]).sum(-1)
        cc = (oc * oc).sum(-1) - r[None] ** 2
        disc = b * b - cc
        t = -b - torch.sqrt(disc.clamp(min=0))
        t = torch.where((disc > 0) & (t > 0), t, torch.full_like(t, math.inf))
        tmin, idx = t.min(-1)
        out = torch.ones(o.shape[0], 3, dtype=torch.float64, device=o.device)
        hit = torch.isfinite(tmin)
        out[hit] = rgb[idx[hit]]
        if self.texture_freq:  # a surface pattern in world space: detail for the fine hash levels
            x = o[hit] + tmin[hit, None] * dn[hit]
            f = self.texture_freq
            pat = torch.sin(f * x[:, 0]) * torch.sin(f * x[:, 1]) * torch.sin(f * x[:, 2])
            out[hit] = (out[hit] + 0.3 * pat[:, None] * torch.tensor([1.0, -0.6, 0.8], dtype=out.dtype,
                                                                     device=out.device)).clamp(0, 1)
        return out.float()

    def density_grid(self, G=128, cascades=1):
        """Occupancy prior (density 100 inside balls, 0 elsewhere) in the reference's Morton order."""
        from . import synthetic
        return synthetic.balls_to_grid(self.c.numpy(), self.r.numpy(), G=G, cascades=cascades)


def ball_scene_views(scene, n_views, W, focal, radius=1.5, seed=0, device="cpu"):
    """n_views cameras on a sphere looking at the origin (synthetic.camera_poses), W x W pinhole
    intrinsics, ground-truth images rendered analytically on `device`: (images (n, W*W, 3),
    poses (n,3,4), directions (W*W, 3), K) -- images on `device`, the rest on the host."""
    from . import synthetic
    poses = synthetic.camera_poses(n_cams=n_views, seed=seed, radius=radius)
    K = torch.tensor([[focal, 0, W / 2], [0, focal, W / 2], [0, 0, 1]], dtype=torch.float32)
    dirs = get_ray_directions(W, W, K)
    dd = dirs.to(device)
    imgs = []
    for p in poses:
        o, d = get_rays(dd, p.to(device))
        imgs.append(scene.render(o, d))
    return torch.stack(imgs), poses, dirs, K

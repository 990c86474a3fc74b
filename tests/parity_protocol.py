"""The short-horizon training-parity protocol (BASELINE config 1 shape: 64x64 views, 256 rays per
batch), shared by tests/golden/make_parity_train.py (which drives the REFERENCE's own render /
NeRFLoss with the CPU oracle injected, in the build container) and tests/test_gpu_parity_train.py
(which drives this repo's fused training step on the GPU).  Everything both sides consume is made
here, deterministically, on the host: the analytic scene and its views, every step's ray batch and
march perturbation, the occupancy bitfield and the initial weights.

Deliberate simplifications (identical on both sides): the occupancy grid is the scene's exact ball
union, held fixed (the refresh cadence is covered by its own bit-exact tests); the cosine schedule
(train.py:136-142: CosineAnnealingLR(T_max=num_epochs-1, eta_min=lr/100), stepped once per epoch)
runs over EPOCHS short epochs of STEPS_PER_EPOCH steps instead of 30 of 1000, so a run ends at the
schedule's small final rate, where its held-out PSNR no longer swings with the last few batches.
"""
import math
import os

import torch

from mfnerf import data, engine, synthetic

W = 64                      # config 1: Lego 64x64 (--downsample 0.08)
FOCAL = 0.5 * W / math.tan(0.5 * 0.6911112)  # the Lego field of view
N_TRAIN = 40
N_TEST = int(os.environ.get("MFNERF_PARITY_TEST_VIEWS", 16))
N_RAYS = 256                # config 1's batch
EPOCHS = int(os.environ.get("MFNERF_PARITY_EPOCHS", 10))
STEPS_PER_EPOCH = int(os.environ.get("MFNERF_PARITY_EPOCH_STEPS", 200))
STEPS = EPOCHS * STEPS_PER_EPOCH
LR = 1e-2
INIT_SEED = 1337
LOG_EVERY = 20


def lr_at(step):
    """train.py:136-142's per-epoch cosine schedule at global step `step`."""
    T_max, eta_min = EPOCHS - 1, LR * 0.01
    e = min(step // STEPS_PER_EPOCH, T_max)
    return LR if T_max <= 0 else eta_min + (LR - eta_min) * (1 + math.cos(math.pi * e / T_max)) / 2


def config():
    """The Lego defaults (opt.py): Hash L16 F2 T2^19, N_min 16, N_max 2048, rgb 64x2, scale 0.5."""
    return engine.StepConfig(n_rays=N_RAYS, lr=LR)


def scene():
    sc = data.BallScene.matching_grid(seed=0)  # the balls of synthetic.ball_density_grid()
    train = data.ball_scene_views(sc, N_TRAIN, W, FOCAL, seed=3)
    test = data.ball_scene_views(sc, N_TEST, W, FOCAL, seed=7)
    return train, test


def density_grid():
    return synthetic.ball_density_grid()


def batch(train, step, seed=0):
    """(rays_o, rays_d, rgb) of step `step` of run `seed`: a random pixel of a random training view
    per ray (datasets/base.py:22-35 'all_images'), rays as ray_utils.get_rays builds them."""
    imgs, poses, dirs, _ = train
    g = torch.Generator().manual_seed(10000 + step + 1000003 * seed)
    img = torch.randint(imgs.shape[0], (N_RAYS,), generator=g)
    pix = torch.randint(imgs.shape[1], (N_RAYS,), generator=g)
    c2w = poses[img]
    rays_d = (dirs[pix][:, None, :] @ c2w[:, :, :3].transpose(1, 2))[:, 0].contiguous()
    rays_o = c2w[:, :, 3].contiguous()
    return rays_o, rays_d, imgs[img, pix].contiguous()


def noise(step, seed=0):
    """The march perturbation of step `step` of run `seed` (custom_functions.py:83, torch.rand_like)."""
    return torch.rand(N_RAYS, generator=torch.Generator().manual_seed(20000 + step + 1000003 * seed))


def init_params(cfg):
    """(xyz_encoder.params = [xyz MLP | table], rgb_net.params) in tcnn's layout, fp32, host."""
    from mfnerf.field import XYZ_NET_PARAMS, rgb_net_params
    from mfnerf.grid import GridLayout
    b = float(math.exp(math.log(cfg.N_max * cfg.scale / cfg.N_min) / (cfg.L - 1)))
    lay = GridLayout(cfg.L, cfg.F, cfg.log2_T, cfg.N_min, b, cfg.grid, cfg.N_tables)
    n_rgb = rgb_net_params(cfg.rgb_width)
    n_params = XYZ_NET_PARAMS + n_rgb + lay.n_params
    p = engine.init_params(cfg, n_params, n_params, INIT_SEED)
    xyz = torch.cat([p[:XYZ_NET_PARAMS], p[XYZ_NET_PARAMS + n_rgb:n_params]])
    return xyz, p[XYZ_NET_PARAMS:XYZ_NET_PARAMS + n_rgb].clone()


def psnr(pred, gt):
    return float(-10.0 * torch.log10(((pred.float() - gt.float()) ** 2).mean()))

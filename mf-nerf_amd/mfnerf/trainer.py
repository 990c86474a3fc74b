"""train.py's NeRFSystem (train.py:53-245) on the fused engine: the training-harness pieces around
the step.

* occupancy cadence -- a refresh every 16 steps, all cells during the first 256 steps
  (train.py:61-62,164-168), erode for colmap scenes; mark_invisible_cells once at the start
  (train.py:154-157);
* learning rate -- CosineAnnealingLR(T_max=num_epochs-1, eta_min=lr*0.01), stepped per epoch of
  1000 steps (train.py:136-142, datasets/base.py:17-20), held on the device (Adam reads it);
* fp16 loss scaling -- PL precision=16 (train.py:287) = torch GradScaler: the MLP backward runs in
  fp16 at the dynamic loss scale (init 2^16, x2 after 2000 clean steps, x0.5 on an overflow) and
  un-scales inside the kernel; a step whose gradient is not finite is skipped.  Deviation: tcnn
  also multiplies the MLP backward by its own fixed loss_scale of 128, so the reference's fp16
  backward runs at 128x the GradScaler's scale; here field_bw runs at the GradScaler's scale alone,
  so overflow/backoff dynamics start from a 128x lower effective scale (skip-count parity is
  unpinned: the parity fixtures come from an fp32 reference and assert zero skips).  All of it on the
  device (mfnerf_field_bw's non-finite flag and device scale, the optimizer pass's last workgroup
  running GradScaler.update(); mfnerf_amp_state) -- no host synchronisation;
* metrics -- train loss / PSNR / rm_s (train.py:178-189), test PSNR with the test-time renderer
  (train.py:197-206), both read back only every `log_every` steps;
* checkpoints -- the reference's state-dict keys (model.xyz_encoder.params, model.rgb_net.params,
  model.density_bitfield, ...; utils.py:4-39), loaded with torch.load(weights_only=True).
The data step is GPU-resident (mfnerf.data.DeviceDataset): no DataLoader, no host copies.
"""
import math
from dataclasses import dataclass

import torch

from . import engine

WARMUP_STEPS = 256     # train.py:61
UPDATE_INTERVAL = 16   # train.py:62


@dataclass
class HParams:
    """The opt.py fields the training step reads (opt.py:7-95), with the reference's defaults."""
    dataset_name: str = "nsvf"
    scale: float = 0.5
    distortion_loss_w: float = 0.0
    batch_size: int = 8192
    ray_sampling_strategy: str = "all_images"
    num_epochs: int = 30
    lr: float = 1e-2
    random_bg: bool = False
    grid: str = "Hash"
    L: int = 16
    F: int = 2
    T: int = 19
    N_min: int = 16
    N_max: int = 2048
    N_tables: int = 1
    rgb_channels: int = 64
    rgb_layers: int = 2
    seed: int = 1337
    steps_per_epoch: int = 1000  # len(train dataset) (datasets/base.py:17-20)


def cosine_lr(epoch, hp: HParams):
    """CosineAnnealingLR(opt, T_max=num_epochs-1, eta_min=lr*0.01) after `epoch` scheduler steps."""
    T_max, lr, eta_min = hp.num_epochs - 1, hp.lr, hp.lr * 0.01
    if T_max <= 0:
        return lr
    return eta_min + (lr - eta_min) * (1 + math.cos(math.pi * min(epoch, T_max) / T_max)) / 2


def psnr(pred, gt):
    return float(-10.0 * torch.log10(((pred - gt) ** 2).mean()))


class Trainer:
    def __init__(self, hp: HParams, train, device="cuda", rank=0, world=1, graphs=True):
        if hp.random_bg:
            raise NotImplementedError("the fused step trains with a fixed background (random_bg off)")
        if hp.rgb_layers != 2:
            raise NotImplementedError("the fused field head implements rgb_layers=2")
        self.hp, self.train = hp, train
        cfg = engine.StepConfig(n_rays=hp.batch_size, scale=hp.scale, L=hp.L, F=hp.F, log2_T=hp.T, N_min=hp.N_min,
                                N_max=hp.N_max, grid=hp.grid, N_tables=hp.N_tables, rgb_width=hp.rgb_channels,
                                lr=hp.lr, lambda_distortion=hp.distortion_loss_w)
        self.step = engine.TrainStep(cfg, device=device, seed=hp.seed)
        if world > 1:
            self.step.shard_optimizer(rank, world)
        self.step.attach_dataset(train)
        self.graphs = graphs
        self.global_step = 0
        self.count_grid = None
        if train.K is not None and train.img_wh is not None:  # on_train_start (train.py:154-157)
            self.mark_invisible_cells(train.K, train.poses, train.img_wh)

    # ---------------------------------------------------------------- occupancy
    @torch.no_grad()
    def mark_invisible_cells(self, K, poses, img_wh):
        from .networks import _meshgrid3d, mark_invisible_cells
        st = self.step
        coords = _meshgrid3d(st.G, device=st.dev)
        self.count_grid = mark_invisible_cells(st.density_grid, coords, st.cfg.scale, K.to(st.dev),
                                               poses.to(st.dev), img_wh)

    def refresh_occupancy(self):
        """train.py:164-168 for the current global step."""
        erode = self.hp.dataset_name == "colmap"
        self.step.update_density_grid(warmup=self.global_step < WARMUP_STEPS,
                                      count_grid=self.count_grid if erode else None, seed=self.hp.seed)

    # ---------------------------------------------------------------- steps
    def training_step(self):
        st = self.step
        if self.global_step % UPDATE_INTERVAL == 0:
            self.refresh_occupancy()
        # the next step's march may start now unless the next step begins with a refresh
        prefetch = (self.global_step + 1) % UPDATE_INTERVAL != 0
        if self.graphs:
            if st.graphs is None:
                st.run()  # lazy init outside capture
                st.capture()
            else:
                st.replay(prefetch=prefetch)
        else:
            st.run()
        self.global_step += 1

    def fit(self, epochs=None, steps=None, log_every=100, log=None):
        """Train for `epochs` epochs (default hp.num_epochs) of hp.steps_per_epoch steps, or for
        `steps` steps; returns the logged history (list of dicts)."""
        hp = self.hp
        total = steps if steps is not None else (epochs or hp.num_epochs) * hp.steps_per_epoch
        hist = []
        for _ in range(total):
            if self.global_step % hp.steps_per_epoch == 0:
                self.step.set_lr(cosine_lr(self.global_step // hp.steps_per_epoch, hp))
            self.training_step()
            if log_every and self.global_step % log_every == 0:
                m = self.train_metrics()
                hist.append(m)
                if log:
                    log(m)
        return hist

    @torch.no_grad()
    def train_metrics(self):
        """train.py:178-189 for the last step: loss, PSNR of the batch, rm_s."""
        st = self.step
        b = st.last_batch
        bg = 1.0 if st.cfg.scale <= 0.5 else 0.0
        preds = [t.rgb + bg * (1 - t.opacity)[:, None] for t in st.parts]
        pred = torch.cat(preds)
        return {"step": self.global_step, "loss": float(st.loss_sum), "psnr": psnr(pred, b.rgb),
                "rm_s": float(st.live_samples()) / st.cfg.n_rays,
                "lr": float(st.lr_dev), "skipped": st.skipped_steps(),
                # records the partitioned table-gradient scatter could not place in its slots so far
                # (added by integer atomics instead: same sums, slower)
                "overflow_records": st.overflow_records()}

    # ---------------------------------------------------------------- evaluation / checkpoints
    def to_ngp(self):
        """An mfnerf.networks.NGP holding this trainer's current weights and occupancy."""
        from .networks import NGP
        st, hp = self.step, self.hp
        m = NGP(scale=hp.scale, hparams=hp).to(st.dev)
        self._store_into(m)
        return m

    @torch.no_grad()
    def _store_into(self, m):
        st = self.step
        p = st.full_params()
        n_net = engine.XYZ_NET_PARAMS
        m.xyz_encoder.params.copy_(torch.cat([p[:n_net], p[st.off_table:st.n_params]]))
        m.rgb_net.params.copy_(p[st.off_rgb:st.off_table])
        m.density_grid.copy_(st.density_grid)
        m.density_bitfield.copy_(st.bitfield)

    @torch.no_grad()
    def evaluate(self, images, poses, directions, chunk=None):
        """Mean test PSNR over views (train.py:197-206): the test-time renderer (rendering.py:46-118)
        on every pixel of each (images[i], poses[i]) view; also returns the per-view values."""
        from .data import get_rays
        from .rendering import render
        model = self.to_ngp()
        dev = self.step.dev
        dirs = directions.to(dev)
        vals = []
        for img, pose in zip(images, poses):
            o, d = get_rays(dirs, pose.to(dev))
            kw = {"test_time": True}
            if self.hp.scale > 0.5:
                kw["exp_step_factor"] = 1 / 256
            res = render(model, o, d, **kw)
            vals.append(psnr(res["rgb"].float(), img.to(dev)))
        return sum(vals) / len(vals), vals

    def state_dict(self):
        """The reference's keys (NeRFSystem.state_dict -> 'model.*'; utils.py:4-39)."""
        m = self.to_ngp()
        sd = {"model." + k: v.detach().cpu() for k, v in m.state_dict().items()}
        sd["poses"] = self.train.poses.detach().cpu()
        return sd

    def save(self, path):
        torch.save({"state_dict": self.state_dict()}, path)

    @torch.no_grad()
    def load(self, path):
        """Load a checkpoint written by save() or by the reference (utils.load_ckpt semantics:
        'model.'-prefixed keys of a Lightning 'state_dict'), executing nothing from the file."""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        sd = ck.get("state_dict", ck)
        st = self.step
        n_net = engine.XYZ_NET_PARAMS
        xyz = sd["model.xyz_encoder.params"].float().to(st.dev)
        rgb = sd["model.rgb_net.params"].float().to(st.dev)
        if xyz.numel() != n_net + st.layout.n_params or rgb.numel() != st.n_rgb:
            raise ValueError("checkpoint does not match this model's configuration")
        st.params[:n_net].copy_(xyz[:n_net])
        st.params[st.off_table:st.n_params].copy_(xyz[n_net:])
        st.params[st.off_rgb:st.off_table].copy_(rgb)
        st.p16.copy_(st.params.half())
        st._pack()
        # the reference's slim checkpoints carry no optimizer state: it loads the weights before it
        # builds FusedAdam (train.py:129,136), so the next update is Adam's step 1 with fresh moments
        st.m.zero_()
        st.v.zero_()
        st.step_dev.zero_()
        st.adam_step = 0
        # ... and a fresh GradScaler (PL precision=16 builds it at init 2^16, train.py:287): the
        # loss scale, growth tracker and skip count do not carry over
        st.reset_loss_scale()
        if "model.density_grid" in sd:
            st.density_grid.copy_(sd["model.density_grid"].to(st.dev))
        if "model.density_bitfield" in sd:
            st.bitfield.copy_(sd["model.density_bitfield"].to(st.dev))

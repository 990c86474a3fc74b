"""The fused MI355X training step: one NeRF training iteration of the reference's hot path
(train.py:164-190 -> rendering.py:121-163 -> losses.py:47-60 -> backward -> FusedAdam) as a
fixed set of gfx950 kernels with every intermediate resident in HBM and the sample counts kept on
the device (no host synchronisation, so a step is capturable in HIP graphs).

Parts.  The batch's rays are split into `n_parts` equal, independent ray ranges ("parts"): each
part is marched into its own sample buffers (own device counter, own rays_a) and runs its own
encode -> field -> composite -> loss -> backward chain; the loss of every part is normalised by the
FULL batch size (mfnerf_nerf_loss n_mean), so the parts' gradients add up to exactly the
full batch's.  Parts exist so that the chain of part p+1 (MFMA/VALU work) runs on another stream
while part p's table-gradient scatter (grid_bw, bound by memory-side atomics) keeps the memory
system busy.  n_parts = 1 is the plain single-batch step.

Buffers are sized once for the worst case (n_rays * MAX_SAMPLES samples, as the reference's
raymarching_train does); kernels that run per sample read the live count from their part's
`counter[0]` and grid-stride over it.  Parameters live in one flat fp32 vector
    params = [xyz MLP (3072) | rgb MLP (7168) | grid table (L*F*entries)]
so Adam is one launch and the gradient zeroing one memset; an fp16 mirror of the whole vector is
refreshed by the same Adam pass and is what the grid kernels gather from.
Multi-GPU: run/replay(exchange=dp.allreduce_mean_) all-reduces `grads` between backward and Adam.
"""
import ctypes
import math
from dataclasses import dataclass

import numpy as np
import torch

from . import synthetic
from ._lib import AdamFused, call, load, ptr, stream
from .field import XYZ_NET_PARAMS, rgb_net_params
from .grid import GridLayout

MAX_SAMPLES = 1024
GATE_TIMEOUT_US = 2000  # a gated march starts anyway after this long (gate.hip)
NEAR_DISTANCE = 0.01
SQRT3 = 3 ** 0.5


@dataclass
class StepConfig:
    n_rays: int = 8192
    scale: float = 0.5
    L: int = 16
    F: int = 2
    log2_T: int = 19
    N_min: int = 16
    N_max: int = 2048
    grid: str = "Hash"
    N_tables: int = 1
    rgb_width: int = 64
    lr: float = 1e-2
    eps: float = 1e-15
    lambda_opacity: float = 1e-3
    lambda_distortion: float = 0.0  # NeRFLoss(lambda_distortion) = --distortion_loss_w (losses.py:40-60)
    T_threshold: float = 1e-4
    max_samples: int = MAX_SAMPLES
    n_parts: int = 1
    skip_nonfinite: bool = True  # GradScaler semantics: no optimizer step on an inf/nan gradient
    # PL precision=16 (train.py:287) = torch GradScaler defaults: init 2^16, x2 after 2000 clean steps,
    # x0.5 on an overflow; dynamic_loss_scale=False keeps a fixed 2^(floor(log2 n_rays)-2) instead
    dynamic_loss_scale: bool = True
    loss_scale: float = 65536.0
    growth_interval: int = 2000
    fixed_point_grid: bool = True  # table gradient by int32 fixed-point atomics (n_parts == 1)
    # ... of the hashed tables by partitioned LDS sums (mfnerf_grid_encode_bw_binned); False keeps the
    # memory-side-atomic scatter (the layouts the partitions do not support take it anyway)
    binned_grid: bool = True
    # the binned scatter's record slots are sized for this many samples per ray (the capacity is
    # max_samples = 1024 per ray; trained scenes march ~60): a step marching more than ~3x this
    # (the first steps, before the occupancy grid is pruned) overflows slots, whose extra records
    # are added by integer atomics (same sums, slower)
    bin_samples_per_ray: int = 128


@dataclass
class Batch:
    rays_o: torch.Tensor
    rays_d: torch.Tensor
    rgb: torch.Tensor


class _State:
    @property
    def loss_sum(self):
        """The step's loss (device scalar): the sum of the loss partial sums."""
        return self.loss_parts.sum()


def _packed_batch(buf):
    """Batch whose tensors are views into one (3, N, 3) buffer (rays_o, rays_d, rgb)."""
    b = Batch(buf[0], buf[1], buf[2])
    b.buf = buf
    return b


def init_params(c: StepConfig, n_params, n_alloc, seed):
    """The flat initial parameters [xyz MLP | rgb MLP | table] (host tensor, n_alloc long, zero
    padding): tcnn's init -- Xavier-uniform per MLP matrix, table U(-1e-4, 1e-4) -- from a seeded
    generator, so a CPU restatement of the step can start from the very same weights."""
    g = torch.Generator().manual_seed(seed)
    p = torch.zeros(n_alloc)
    off = 0
    for o, k in [(64, 32), (16, 64), (c.rgb_width, 32), (c.rgb_width, c.rgb_width), (16, c.rgb_width)]:
        s = math.sqrt(6.0 / (o + k))  # tcnn Xavier-uniform per matrix
        p[off:off + o * k].uniform_(-s, s, generator=g)
        off += o * k
    p[off:n_params].uniform_(-1e-4, 1e-4, generator=g)  # tcnn grid init
    return p


class TrainStep:
    def __init__(self, cfg: StepConfig, device="cuda", seed=0):
        self.cfg = cfg
        self.dev = torch.device(device)
        load()
        c = cfg
        if c.n_parts < 1 or c.n_rays % c.n_parts:
            raise ValueError(f"n_rays={c.n_rays} must split into n_parts={c.n_parts} equal parts")
        self.cascades = max(1 + int(np.ceil(np.log2(2 * c.scale))), 1)
        self.G = 128
        b = float(np.exp(np.log(c.N_max * c.scale / c.N_min) / (c.L - 1)))
        self.layout = GridLayout(c.L, c.F, c.log2_T, c.N_min, b, c.grid, c.N_tables)
        self.desc = self.layout.desc()
        self.n_rgb = rgb_net_params(c.rgb_width)
        self.off_rgb = XYZ_NET_PARAMS
        self.off_table = XYZ_NET_PARAMS + self.n_rgb
        self.n_params = self.off_table + self.layout.n_params
        # flat buffers are padded (zeros, never updated) so any power-of-two world size shards them
        # into float4-aligned equal slices (shard_optimizer)
        self.n_alloc = -(-self.n_params // 16384) * 16384
        s32 = np.float32(c.scale)
        self.x_min, self.x_range = float(-s32), float(np.float32(s32) - np.float32(-s32))

        dev = self.dev
        self.params = init_params(c, self.n_params, self.n_alloc, seed).to(dev)
        self.grads = torch.zeros(self.n_alloc, device=dev)
        self.m = torch.zeros(self.n_alloc, device=dev)
        self.v = torch.zeros(self.n_alloc, device=dev)
        self.p16 = self.params.half()
        self.shard = None  # (rank, lo, hi) once shard_optimizer() is on
        # mfnerf_amp_state: [non-finite flag, skipped steps, scale, growth tracker, growth interval,
        # growth factor, backoff factor, ticket] (include/mfnerf.h)
        self.finite_status = torch.zeros(8, dtype=torch.int32, device=dev)
        self.reset_loss_scale()
        self.packed = torch.empty(load().mfnerf_field_packed_bytes(c.rgb_width) // 2, dtype=torch.float16,
                                  device=dev)
        self._pack()
        self.adam_step = 0                                            # host mirror
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)  # Adam's t, bumped on the device
        self.lr_dev = torch.full((1,), float(c.lr), dtype=torch.float32, device=dev)
        self.graphs = None
        self.samples_marched = torch.zeros(1, dtype=torch.int64, device=dev)

        # scene bounding box (networks.py:18-23) and occupancy
        self.center = torch.zeros(1, 3, device=dev)
        self.half_size = torch.full((1, 3), c.scale, device=dev)
        self.density_grid = torch.zeros(self.cascades, self.G ** 3, device=dev)
        self.bitfield = torch.zeros(self.cascades * self.G ** 3 // 8, dtype=torch.uint8, device=dev)

        N = c.n_rays
        self.n_parts = c.n_parts
        self.Np = N // c.n_parts                      # rays per part
        self.cap_p = self.Np * c.max_samples          # sample capacity per part
        self.cap = N * c.max_samples
        self.parts = [self._part_buffers(q) for q in range(c.n_parts)]
        self.mbuf = [self._march_buffers()]  # a second set is added by capture() (pipelined march)
        # the step's loss as partial sums: one per 4 rays of each part (written by the fused
        # compositing kernel) + 64 accumulated slots (unfused path: NeRFLoss atomics, distortion)
        self._nb_part = -(-self.Np // 4)
        self._level_l1 = torch.zeros(c.L, dtype=torch.float32, device=dev)
        self.loss_parts = torch.zeros(c.n_parts * self._nb_part + 64, dtype=torch.float32, device=dev)
        self._loss_acc = self.loss_parts[c.n_parts * self._nb_part:]
        self.state = _State()
        self._use(self.mbuf[0])
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed + 1)
        # static fp16 backward scale: per-sample grads are O(1/n_rays); 2^(floor(log2 N)-2) keeps them
        # normal.  With the dynamic scale (default) field_bw reads amp.scale on the device instead.
        self.grad_scale = float(2.0 ** max(0, int(math.floor(math.log2(N))) - 2))
        self._primed = False
        self._stale_pack = False  # a one-graph data-parallel replay left `packed` one update behind
        self.dataset = None

    def reset_loss_scale(self, scale=None):
        """(Re)initialise the device GradScaler state (mfnerf_amp_state) from the config."""
        c = self.cfg
        a = torch.zeros(8, dtype=torch.int32)
        af = a.view(torch.float32)
        af[2] = float(c.loss_scale if scale is None else scale)
        a[4] = int(c.growth_interval) if c.dynamic_loss_scale else 0
        af[5], af[6] = 2.0, 0.5
        self.finite_status.copy_(a.to(self.dev))

    def _amp_on(self):
        """GradScaler bookkeeping on the device: the skip (and, dynamic, the scale update)."""
        return self.cfg.skip_nonfinite or self.cfg.dynamic_loss_scale

    def _amp_ptr(self):
        return ptr(self.finite_status) if self._amp_on() else None

    def loss_scale(self):
        """The loss scale the next backward uses (host read)."""
        if not self.cfg.dynamic_loss_scale:
            return self.grad_scale
        return float(self.finite_status.view(torch.float32)[2])

    def attach_dataset(self, ds):
        """Draw every step's batch on the device from ds (mfnerf.data.DeviceDataset): run() and
        replay() then take no batch; inside graphs the draw is part of the march graph."""
        self.dataset = ds
        self._sampled = _packed_batch(torch.zeros(3, self.cfg.n_rays, 3, device=self.dev))
        self.graphs = None

    # ---------------------------------------------------------------- buffers
    def _part_buffers(self, q):
        """Per-part sample/ray state of the chain (features, field outputs, compositing, grads)."""
        c, dev, Np, cap = self.cfg, self.dev, self.Np, self.cap_p
        f32 = dict(dtype=torch.float32, device=dev)
        t = _State()
        # encoded features as level planes (L, cap) of half2 (mfnerf_grid_encode_fw_planar)
        t.feat = torch.empty(c.L, cap, c.F, dtype=torch.float16, device=dev)
        t.sigma = torch.empty(cap, **f32)
        t.rgb_s = torch.empty(cap, 3, **f32)
        t.total = torch.empty(Np, dtype=torch.int64, device=dev)
        t.opacity = torch.empty(Np, **f32)
        t.depth = torch.empty(Np, **f32)
        t.rgb = torch.empty(Np, 3, **f32)
        t.ws = torch.empty(cap, **f32)
        t.dL_drgb = torch.empty(Np, 3, **f32)
        t.dL_dop = torch.empty(Np, **f32)
        t.zeros_ray = torch.zeros(Np, **f32)       # dL/ddepth (unused by the loss; unfused path)
        if c.lambda_distortion > 0:                # losses.py:6-37 + 55-58
            t.dist_loss = torch.empty(Np, **f32)
            t.ws_incl = torch.empty(cap, **f32)
            t.wts_incl = torch.empty(cap, **f32)
            t.dL_ddist = torch.full((Np,), c.lambda_distortion / c.n_rays, **f32)  # d(lambda*mean)/dloss_r
            t.dL_dws = torch.empty(cap, **f32)
        t.dsig = torch.empty(cap, **f32)
        t.drgb_s = torch.empty(cap, 3, **f32)
        t.dfeat = torch.empty(cap, c.L * c.F, **f32)
        t.field_ws = torch.empty(load().mfnerf_field_bw_workspace(cap, c.rgb_width) // 4, **f32)
        if self._binned():
            nb = load().mfnerf_grid_encode_bw_binned_workspace(self.desc, self._bin_slots())
        else:
            nb = load().mfnerf_grid_encode_bw_workspace(self.desc)
        t.grid_ws = torch.zeros(max(16, nb) // 4, **f32)
        # parts > 0 accumulate their MLP weight grads privately (field_bw's slab sum is a plain +=)
        t.mlp_grad = self.grads[:self.off_table] if q == 0 else torch.zeros(self.off_table, **f32)
        return t

    def _march_buffers(self):
        """One set of ray-march outputs: AABB hits and noise for the whole batch, samples per part."""
        c, N, dev = self.cfg, self.cfg.n_rays, self.dev
        f32 = dict(dtype=torch.float32, device=dev)
        m = _State()
        m.hit_cnt = torch.empty(N, dtype=torch.int32, device=dev)
        m.hits = torch.empty(N, 1, 2, **f32)
        m.hits_t = m.hits[:, 0]
        m.hits_idx = torch.empty(N, 1, dtype=torch.int64, device=dev)
        m.noise = torch.empty(N, **f32)
        m.counters = torch.zeros(c.n_parts, 2, dtype=torch.int32, device=dev)  # per part (samples, rays)
        m.part = []
        for q in range(c.n_parts):
            t = _State()
            t.rays_a = torch.empty(self.Np, 3, dtype=torch.int64, device=dev)
            t.xyzs = torch.empty(self.cap_p, 3, **f32)
            t.dirs = torch.empty(self.cap_p, 3, **f32)
            t.deltas = torch.empty(self.cap_p, **f32)
            t.ts = torch.empty(self.cap_p, **f32)
            t.counter = m.counters[q]
            ws_bytes = load().mfnerf_raymarching_train_workspace(self.Np, c.max_samples)
            t.march_ws = torch.empty(max(16, ws_bytes), dtype=torch.uint8, device=dev)
            m.part.append(t)
        return m

    def _use(self, mb):
        """state.noise / state.counters / state.loss_sum of the step being run (inspection)."""
        st = self.state
        st.noise, st.counters, st.loss_parts, st.march = mb.noise, mb.counters, self.loss_parts, mb
        st.parts = self.parts

    @property
    def loss_sum(self):
        return self.loss_parts.sum()

    def live_samples(self):
        """Device scalar: samples marched by the current step (sum over parts)."""
        return self.state.counters[:, 0].sum()

    def gather_march(self):
        """(rays_a (N,3) i64 with global starts, xyzs (n,3), dirs, deltas, ts) of the current step,
        concatenated over parts in ray order -- host-synchronising, for tests and smoke()."""
        mb = self.state.march
        ra, xs, ds, dl, ts = [], [], [], [], []
        base = 0
        for q, t in enumerate(mb.part):
            n = int(mb.counters[q, 0])
            r = t.rays_a.clone()
            r[:, 0] += q * self.Np
            r[:, 1] += base
            ra.append(r)
            xs.append(t.xyzs[:n]); ds.append(t.dirs[:n]); dl.append(t.deltas[:n]); ts.append(t.ts[:n])
            base += n
        return torch.cat(ra), torch.cat(xs), torch.cat(ds), torch.cat(dl), torch.cat(ts)

    # ---------------------------------------------------------------- data
    def make_batches(self, k, seed=0):
        """k synthetic Lego-like ray batches (mfnerf.synthetic), resident on the device; each is
        packed in one (3, N, 3) buffer (rays_o, rays_d, rgb) so replay() refreshes with one copy."""
        poses = synthetic.camera_poses(seed=seed)
        out = []
        for i in range(k):
            o, d = synthetic.random_rays(self.cfg.n_rays, poses, seed=seed * 1000 + i)
            dn = d / d.norm(dim=1, keepdim=True)
            gt = 0.5 + 0.5 * torch.sin(3 * dn + torch.tensor([0.0, 1.0, 2.0]))  # smooth view-dependent target
            out.append(_packed_batch(torch.stack([o, d, gt.float()]).to(self.dev)))
        return out

    def set_occupancy(self, density_grid):
        """Install a (C, G^3) density grid and pack it with the reference's threshold."""
        self.density_grid.copy_(density_grid.to(self.dev))
        thr = 0.01 * MAX_SAMPLES / SQRT3
        call("mfnerf_packbits", ptr(self.density_grid), self.bitfield.numel(), thr, None, ptr(self.bitfield), stream())

    def _pack(self):
        """MFMA weight blob from the fp16 compute copy (the fp16 values packing the fp32 master
        would produce), so it works on every rank when the fp32 master is sharded."""
        call("mfnerf_field_pack_weights_f16", ptr(self.p16), ptr(self.p16[self.off_rgb:]), self.cfg.rgb_width,
             ptr(self.packed), stream())

    def _flush_pack(self):
        """Repack if a one-graph data-parallel replay deferred it: that path's Adam runs after the
        collective and the next dp_pre graph starts with the repack, so until then `packed` is one
        update behind.  Everything else that reads `packed` (an eager step, the occupancy refresh,
        the per-stage graphs) calls this first."""
        if self._stale_pack:
            pg = (self.graphs or {}).get("pack")
            pg.replay() if pg is not None else self._pack()
            self._stale_pack = False

    def shard_optimizer(self, rank, world, force=False):
        """Data parallel with a sharded optimizer (mfnerf.dp.sharded_update): this rank keeps Adam
        state only for its 1/world slice of the flat parameters; the step reduce-scatters the
        gradient, updates the slice and all-gathers the fp16 compute copy.  world 1 is a no-op
        unless force (a one-rank process group running the sharded path, for tests)."""
        if world <= 1 and not force:
            return
        if self.n_alloc % (64 * world):
            raise ValueError(f"world size {world} does not divide the padded parameter count {self.n_alloc}")
        k = self.n_alloc // world
        lo, hi = rank * k, (rank + 1) * k
        self.shard = (rank, lo, hi)
        self.m = torch.zeros(k, device=self.dev)
        self.v = torch.zeros(k, device=self.dev)
        # this rank's slice of the gradient, reduced in place (RCCL in-place reduce-scatter: no
        # second gradient-sized buffer, and a one-rank group's "reduction" is no copy)
        self.g_shard = self.grads[lo:hi]
        self._store_fold_v = None  # (re-derived for the sharded step)
        self.graphs = None  # re-capture with the sharded update

    # ---------------------------------------------------------------- the step
    def _draw(self, batch: Batch, mb):
        """The attached dataset's next batch into `batch`, with the march prologue (AABB + near clamp
        + noise) of mb in the same launch."""
        self.dataset.sample(batch.buf, prep=(self.center, self.half_size, NEAR_DISTANCE, mb.hits, mb.noise))

    def _march(self, batch: Batch, mb, mark, prepped=False, noise=None):
        """AABB + near clamp + noise for the whole batch (unless _draw did it), then one ray march per
        part into mb."""
        c, s = self.cfg, stream()
        N, Np = c.n_rays, self.Np
        if not prepped:
            # rendering.py:27-29 (AABB + near clamp), custom_functions.py:83 (noise)
            call("mfnerf_ray_aabb_intersect", ptr(batch.rays_o), ptr(batch.rays_d), ptr(self.center),
                 ptr(self.half_size), N, 1, 1, ptr(mb.hit_cnt), ptr(mb.hits), ptr(mb.hits_idx), s)
            t1 = mb.hits[:, 0, 0]
            t1.masked_fill_((t1 >= 0) & (t1 < NEAR_DISTANCE), NEAR_DISTANCE)
            if noise is None:
                torch.rand(N, generator=self.gen, device=self.dev, out=mb.noise)
            else:  # a given perturbation (parity tests driving the reference with the same draws)
                mb.noise.copy_(noise)
        mark("prep")
        for q, t in enumerate(mb.part):
            r = slice(q * Np, (q + 1) * Np)
            call("mfnerf_raymarching_train", ptr(batch.rays_o[r]), ptr(batch.rays_d[r]), ptr(mb.hits_t[r]), 2,
                 ptr(self.bitfield), self.cascades, float(c.scale), 0.0 if c.scale <= 0.5 else 1 / 256,
                 ptr(mb.noise[r]), self.G, c.max_samples, Np, self.cap_p, ptr(t.rays_a), ptr(t.xyzs), ptr(t.dirs),
                 ptr(t.deltas), ptr(t.ts), ptr(t.counter), ptr(t.march_ws), s)
        # running total of marched samples (rm_s without a read on the step's critical path: in the
        # graphs this runs on the march's side stream)
        # one kernel on the side chain for one part (a slice + reduce + add otherwise)
        self.samples_marched.add_(mb.counters[0, 0] if self.n_parts == 1 else mb.counters[:, 0].sum())
        mark("march")

    def _chain(self, batch: Batch, mb, q, mark):
        """Part q: encode -> field -> composite -> loss -> composite bw -> field bw (no grid bw).
        Part 0 also zeroes the gradient (every part's writes come after it)."""
        c, s = self.cfg, stream()
        t, m = self.parts[q], mb.part[q]
        Np, cap = self.Np, self.cap_p
        store_fold = q == 0 and self._store_fold()
        if q == 0:
            if self.shard is not None and not store_fold:
                # unsharded: the previous Adam pass left it zero; sharded, the binned scatter
                # overwrites the partitioned tables, so only the values before them are zeroed
                self.grads[:self._grad_zero_end()].zero_()
            if c.lambda_distortion > 0:
                self._loss_acc.zero_()
        else:
            t.mlp_grad.zero_()
        call("mfnerf_grid_encode_fw_planar", ptr(m.xyzs), cap, ptr(m.counter), self.x_min, self.x_range, self.desc,
             ptr(self.p16[self.off_table:]), ptr(t.feat), cap, s)
        mark("grid_fw")
        call("mfnerf_field_fw", ptr(t.feat), cap, ptr(m.dirs), cap, ptr(m.counter), ptr(self.packed), c.rgb_width, 0,
             ptr(t.sigma), ptr(t.rgb_s), s)
        mark("field_fw")
        bg = 1.0 if c.scale <= 0.5 else 0.0
        target = ptr(batch.rgb[q * Np:(q + 1) * Np])
        if c.lambda_distortion <= 0:
            # composite fw -> bg blend + NeRFLoss -> composite bw in one wave-per-ray launch
            args = (ptr(t.sigma), ptr(t.rgb_s), ptr(m.deltas), ptr(m.ts), ptr(m.rays_a), Np, cap, c.T_threshold,
                    target, c.n_rays, c.lambda_opacity, bg, bg, bg, ptr(t.total), ptr(t.opacity), ptr(t.depth),
                    ptr(t.rgb), ptr(t.ws), ptr(t.dL_drgb), ptr(t.dL_dop), ptr(t.dsig), ptr(t.drgb_s),
                    ptr(self.loss_parts[q * self._nb_part:]))
            call("mfnerf_composite_train_fused", *args, s)
            mark("composite")
        else:
            call("mfnerf_composite_train_fw", ptr(t.sigma), ptr(t.rgb_s), ptr(m.deltas), ptr(m.ts), ptr(m.rays_a),
                 Np, cap, c.T_threshold, ptr(t.total), ptr(t.opacity), ptr(t.depth), ptr(t.rgb), ptr(t.ws), s)
            call("mfnerf_nerf_loss", ptr(t.rgb), ptr(t.opacity), target, Np, c.n_rays, c.lambda_opacity, bg, bg, bg,
                 ptr(t.dL_drgb), ptr(t.dL_dop), ptr(self._loss_acc), s)
            # losses.py:6-37 + 55-58
            call("mfnerf_distortion_loss_fw", ptr(t.ws), ptr(m.deltas), ptr(m.ts), ptr(m.rays_a), Np, cap,
                 ptr(t.dist_loss), ptr(t.ws_incl), ptr(t.wts_incl), s)
            self._loss_acc[1:2].add_(t.dist_loss.sum() * (c.lambda_distortion / c.n_rays))
            call("mfnerf_distortion_loss_bw", ptr(t.dL_ddist), ptr(t.ws_incl), ptr(t.wts_incl), ptr(t.ws),
                 ptr(m.deltas), ptr(m.ts), ptr(m.rays_a), Np, cap, ptr(t.dL_dws), s)
            mark("composite_fw")
            call("mfnerf_composite_train_bw", ptr(t.dL_dop), ptr(t.zeros_ray), ptr(t.dL_drgb), ptr(t.dL_dws),
                 ptr(t.sigma), ptr(t.rgb_s), ptr(t.ws), ptr(m.deltas), ptr(m.ts), ptr(m.rays_a), ptr(t.opacity),
                 ptr(t.depth), ptr(t.rgb), Np, cap, c.T_threshold, ptr(t.dsig), ptr(t.drgb_s), s)
            mark("composite_bw")
        call("mfnerf_field_bw", ptr(t.feat), cap, ptr(m.dirs), cap, ptr(m.counter), ptr(self.packed), c.rgb_width,
             ptr(t.dsig), ptr(t.drgb_s), 0.0 if c.dynamic_loss_scale else self.grad_scale, ptr(t.dfeat),
             None if store_fold else ptr(t.mlp_grad),
             None if store_fold else ptr(t.mlp_grad[self.off_rgb:]),
             ptr(t.field_ws),
             self._amp_ptr(),
             ptr(self._level_l1) if self._fixed() else None, s)
        if store_fold:  # the fold writes the MLPs' gradient outright (nothing zeroed it)
            call("mfnerf_field_bw_reduce_store", c.rgb_width, ptr(t.field_ws), ptr(t.mlp_grad),
                 ptr(t.mlp_grad[self.off_rgb:]), self._amp_ptr(), s)
        mark("field_bw")

    def _fixed(self):
        """One part: the table gradient is accumulated by int32 fixed-point atomics (per-level scales
        bounded by the L1 norm of dL/dfeat, which field_bw accumulates, so no overflow; the table
        gradient starts at zero because Adam zeroed it); several parts share the gradient and use
        float atomics."""
        return self.n_parts == 1 and self.cfg.fixed_point_grid

    def _binned(self):
        """The fixed-point table gradient by table partitions (one part only, like _fixed), for the
        layouts the partitioned scatter supports; any other layout the reference accepts (opt.py:78,
        e.g. --T 21) keeps the request-shaped fixed-point atomic scatter."""
        if not (self.cfg.n_parts == 1 and self.cfg.fixed_point_grid and self.cfg.binned_grid):
            return False
        if getattr(self, "_bin_supported", None) is None:
            self._bin_supported = load().mfnerf_grid_encode_bw_binned_workspace(self.desc, self._bin_slots()) >= 0
        return self._bin_supported

    def _bin_slots(self):
        """Samples per part the binned scatter's record slots are sized for."""
        return min(self.cap_p, self.Np * max(1, self.cfg.bin_samples_per_ray))

    def _fused_adam_ok(self):
        """The collective-free replayed tail can run the partitioned tables' Adam inside the scatter's
        accumulate (mfnerf_grid_encode_bw_binned_adam + mfnerf_adam_step_fixed_partial)."""
        return self._binned() and self.shard is None and load().mfnerf_grid_binned_first_value(self.desc) >= 0

    def _adam_fused_args(self):
        c = self.cfg
        amp = self._amp_ptr()
        return AdamFused(params=self.params.data_ptr(), m=self.m.data_ptr(), v=self.v.data_ptr(),
                         p16=self.p16.data_ptr(), table_offset=self.off_table, lr=float(c.lr), beta1=0.9,
                         beta2=0.999, eps=float(c.eps), step_dev=self.step_dev.data_ptr(),
                         lr_dev=self.lr_dev.data_ptr(), amp=amp.value if amp is not None else None)

    def _grid_bw(self, mb, q, fuse_adam=False, gate=None):
        """Part q's hash-table gradient scatter (the dominant kernel, alone so it can be timed);
        fuse_adam: with the partitioned tables' Adam step (then _finish_update(partial=True));
        fuse_adam="all": with the whole optimizer step and the MLP repack.  gate (the side stream's
        gate pointer): opened as the scatter starts -- by the dense-level launch's first workgroup
        where the launch takes a gate, else by a signal kernel of its own just before it."""
        t, m = self.parts[q], mb.part[q]
        if gate is not None:
            self._gate_opened += 1
        if self._binned() and fuse_adam == "all":
            self._fused_args = self._adam_fused_args()  # kept alive: graphs capture the call
            call("mfnerf_grid_encode_bw_binned_adam_all", ptr(m.xyzs), self.cap_p, ptr(m.counter), self.x_min,
                 self.x_range, self.desc, ptr(t.dfeat), ptr(self.grads), self.n_alloc, ptr(t.grid_ws),
                 self._bin_slots(), ptr(self._level_l1), ctypes.byref(self._fused_args), ptr(self.step_dev),
                 self._amp_ptr(), ptr(self.packed), self.cfg.rgb_width, gate, stream())
            return
        if gate is not None:
            call("mfnerf_gate_signal", gate, stream())
        if self._binned() and fuse_adam:
            self._fused_args = self._adam_fused_args()  # kept alive: graphs capture the call
            call("mfnerf_grid_encode_bw_binned_adam", ptr(m.xyzs), self.cap_p, ptr(m.counter), self.x_min,
                 self.x_range, self.desc, ptr(t.dfeat), ptr(self.grads[self.off_table:]), ptr(t.grid_ws),
                 self._bin_slots(), ptr(self._level_l1), ctypes.byref(self._fused_args), stream())
            return
        if self._binned():
            # both parts in sequence on this stream: the coarse levels' atomics, then the fine levels'
            # partitioned sums (the two on separate streams inside the graphs measured 1.32 vs
            # 0.87 ms per step: the extra branch slowed every kernel beside it)
            call("mfnerf_grid_encode_bw_binned", ptr(m.xyzs), self.cap_p, ptr(m.counter), self.x_min, self.x_range,
                 self.desc, ptr(t.dfeat), ptr(self.grads[self.off_table:]), ptr(t.grid_ws), self._bin_slots(),
                 ptr(self._level_l1), 3, stream())
            return
        call("mfnerf_grid_encode_bw_scatter", ptr(m.xyzs), self.cap_p, ptr(m.counter), self.x_min, self.x_range,
             self.desc, ptr(t.dfeat), ptr(self.grads[self.off_table:]), ptr(t.grid_ws),
             ptr(self._level_l1) if self._fixed() else None, stream())

    def _store_fold(self):
        """Sharded, one part, partitioned scatter whose float finish overwrites every table value
        before the partitioned tables (they are all dense-prefix values): the weight-gradient fold
        stores instead of adding and the step zeroes no gradient prefix (one fill launch less)."""
        v = getattr(self, "_store_fold_v", None)
        if v is None:
            lib = load()
            n_dw = lib.mfnerf_field_bw_workspace(0, self.cfg.rgb_width) // (4 * lib.mfnerf_field_bw_slab_rows(
                self.cfg.rgb_width))
            v = (self.shard is not None and self.n_parts == 1 and self._binned() and self._fixed()
                 and self.off_table == n_dw
                 and lib.mfnerf_grid_binned_first_value(self.desc) == lib.mfnerf_grid_dense_values(self.desc))
            self._store_fold_v = v
        return v

    def _grad_zero_end(self):
        """Gradient values a step must find zero: all of them, or with the binned scatter only those
        before the partitioned tables (the accumulate stores the rest; overflowed records go through
        the workspace's own words)."""
        if self._binned():
            return self.off_table + load().mfnerf_grid_binned_first_value(self.desc)
        return self.n_alloc

    def _grid_bw_float(self, mb, zero_l1=True, gate=None, shard_flag=None):
        """Data parallel, one part: the table gradient scattered and finished to floats for the
        exchange (binned: the accumulate writes the partitioned tables' floats and one finish pass
        covers the rest, mfnerf_grid_encode_bw_binned_float), level_l1 zeroed after use (zero_l1
        False: the sharded Adam's last workgroup zeroes it, _adam_shard); gate: the side stream's
        gate pointer, opened as the dense-level launch starts (no signal launch of its own);
        shard_flag (flag pointer, shards, shard length): mfnerf_flag_to_shards folded into the
        float finish when it has a table prefix to ride -- returns True when it was."""
        if not self._binned():
            self._grid_bw(mb, 0, gate=gate)
            self._grid_finish(0)
            return False
        t, m = self.parts[0], mb.part[0]
        if gate is not None:
            self._gate_opened += 1
        fold_flag = shard_flag is not None and load().mfnerf_grid_binned_first_value(self.desc) > 0
        fl, fw, fs = shard_flag if fold_flag else (None, 0, 0)
        call("mfnerf_grid_encode_bw_binned_float", ptr(m.xyzs), self.cap_p, ptr(m.counter), self.x_min,
             self.x_range, self.desc, ptr(t.dfeat), ptr(self.grads[self.off_table:]), ptr(t.grid_ws),
             self._bin_slots(), ptr(self._level_l1), gate, fl, fw, fs, self.off_table, stream())
        if zero_l1:
            self._level_l1.zero_()
        return fold_flag

    def _grid_finish(self, q):
        """Fold part q's private copies of the coarse levels / convert the fixed-point sums."""
        call("mfnerf_grid_encode_bw_finish", self.desc, ptr(self.grads[self.off_table:]), ptr(self.parts[q].grid_ws),
             ptr(self._level_l1) if self._fixed() else None, stream())
        if self._fixed():
            self._level_l1.zero_()  # field_bw accumulates it; zeroed once used (also by adam_step_fixed)

    def _reduce_parts(self):
        """Fold parts 1.. MLP weight grads into grads (the table part is already shared)."""
        for t in self.parts[1:]:
            self.grads[:self.off_table].add_(t.mlp_grad)

    def _adam(self, grads, lo, hi, zero_grads):
        """Adam over params[lo:hi] with grads (hi-lo), refreshing p16[lo:hi]; a no-op (but for the
        zeroing) when the step's non-finite flag is up (raised by field_bw, cleared by the call)."""
        c = self.cfg
        call("mfnerf_adam_step", ptr(self.params[lo:hi]), ptr(grads), ptr(self.m), ptr(self.v), ptr(self.p16[lo:hi]),
             hi - lo, float(c.lr), 0.9, 0.999, c.eps, 1.0, 0, ptr(self.step_dev), ptr(self.lr_dev),
             self._amp_ptr(), int(zero_grads), stream())

    def _adam_shard(self):
        """The sharded update after the reduce-scatter with the exchanged non-finite flag read from
        the shard itself and level_l1 zeroed by its last workgroup (mfnerf_adam_step_shard: the
        flag_from_shard launch and the level_l1 fill folded in)."""
        c, (_, lo, hi) = self.cfg, self.shard
        call("mfnerf_adam_step_shard", ptr(self.params[lo:hi]), ptr(self.g_shard), ptr(self.m), ptr(self.v),
             ptr(self.p16[lo:hi]), hi - lo, float(c.lr), 0.9, 0.999, c.eps, 1.0, ptr(self.step_dev), ptr(self.lr_dev),
             self._amp_ptr(), ptr(self._level_l1), self._level_l1.numel(), stream())

    def _finish_update(self, partial=False):
        """Unsharded, no exchange, fixed-point table gradient: the finish (convert) and Adam in one
        pass (mfnerf_adam_step_fixed), then the MLP weight repack.  partial: after a fused
        _grid_bw, only the values before the partitioned tables (all of them if a slot overflowed)."""
        c = self.cfg
        if partial:
            ws = self.parts[0].grid_ws
            ovf = ctypes.c_void_p(ws.data_ptr() + load().mfnerf_grid_encode_bw_binned_flag_offset(
                self.desc, self._bin_slots()))
            call("mfnerf_adam_step_fixed_partial", ptr(self.params), ptr(self.grads), ptr(self.m), ptr(self.v),
                 ptr(self.p16), self.n_alloc, self.off_table, self.desc, ptr(ws), ptr(self._level_l1),
                 float(c.lr), 0.9, 0.999, c.eps, ptr(self.step_dev), ptr(self.lr_dev), self._amp_ptr(),
                 self.off_table + load().mfnerf_grid_binned_first_value(self.desc), ovf, stream())
        else:
            call("mfnerf_adam_step_fixed", ptr(self.params), ptr(self.grads), ptr(self.m), ptr(self.v),
                 ptr(self.p16), self.n_alloc, self.off_table, self.desc, ptr(self.parts[0].grid_ws),
                 ptr(self._level_l1), float(c.lr), 0.9, 0.999, c.eps, ptr(self.step_dev), ptr(self.lr_dev),
                 self._amp_ptr(), stream())
        self._pack()

    def _update(self):
        """Adam over the flat params (+ fp16 mirror, + zeroing the gradient for the next step) +
        MLP weight repack (unsharded)."""
        self._adam(self.grads, 0, self.n_alloc, True)
        self._pack()

    def _shard_adam(self, adam):
        """Sharded: the flag already holds the union over ranks (carried through the
        reduce-scatter, dp.sharded_update), so every rank takes the same decision."""
        adam()

    def full_params(self):
        """The fp32 master parameters (all-gathered over ranks when the optimizer is sharded)."""
        if self.shard is None:
            return self.params
        from . import dp
        full = self.params.clone()
        dp.all_gather_(full, self.shard[0])
        return full

    def overflow_records(self):
        """Records the partitioned scatter could not place in their slots so far (added by integer
        atomics instead; a running total kept by the kernel; host read).  0 without partitions."""
        if not self._binned():
            return 0
        off = load().mfnerf_grid_encode_bw_binned_flag_offset(self.desc, self._bin_slots())
        ws = self.parts[0].grid_ws
        return int(ws.view(torch.int32)[off // 4 + 1])

    def skipped_steps(self):
        """Optimizer steps skipped on non-finite gradients so far (host read)."""
        return int(self.finite_status[1])

    def _optimize(self, exchange, adam=None, pack=None):
        """The update half of a step.  Sharded: reduce-scatter -> Adam on the shard -> all-gather
        fp16 -> repack; else: exchange(grads) (all-reduce, optional) -> Adam -> repack.  adam/pack
        replace the eager launches by graph replays."""
        from . import dp
        self.adam_step += 1
        if self.shard is not None:
            rank, lo, hi = self.shard
            dp.sharded_update(self.grads, self.g_shard, self.p16, rank,
                              adam or (lambda g: self._shard_adam(lambda: self._adam(g, lo, hi, False))),
                              flag=self.finite_status[:1] if self._amp_on() else None)
            (pack or self._pack)()
        else:
            if exchange is not None:
                # the non-finite flag rides the all-reduce: NaN in element 0 when set, read back
                flag = self.finite_status[:1] if self._amp_on() else None
                if flag is not None:
                    call("mfnerf_flag_to_shards", ptr(self.grads), 1, self.n_alloc, ptr(flag), stream())
                exchange(self.grads)
                if flag is not None:
                    call("mfnerf_flag_from_shard", ptr(self.grads), ptr(flag), stream())
            if adam is not None:
                adam(None)
                (pack or (lambda: None))()
            else:
                self._update()

    def run(self, batch: Batch = None, mark=None, exchange=None, optimize=True, noise=None):
        """One training step, eagerly on the current stream, parts in sequence, march buffer set 0.
        mark(name) is called after each stage (bench timing); exchange(grads) runs between backward
        and Adam (the data-parallel all-reduce).  batch=None: drawn from the attached dataset.
        optimize=False stops after the backward and leaves the step's gradient in self.grads (no
        Adam step, no repack; for inspection)."""
        mark = mark or (lambda name: None)
        self._flush_pack()
        mb = self.mbuf[0]
        prepped = batch is None
        if prepped:
            batch = self._sampled
            self._draw(batch, mb)
        self._use(mb)
        self.last_batch = batch
        self._primed = False  # a pipelined replay() must march its own batch next
        self._march(batch, mb, mark, prepped=prepped, noise=noise)
        dp = self.shard is not None or exchange is not None
        for q in range(self.n_parts):
            self._chain(batch, mb, q, mark)
            if dp and self.n_parts == 1:  # the data-parallel step's form (as the captured dp_pre)
                self._grid_bw_float(mb)
                mark("grid_bw")
                mark("grid_finish")
                continue
            self._grid_bw(mb, q)
            mark("grid_bw")
            self._grid_finish(q)
            mark("grid_finish")
        self._reduce_parts()
        if optimize:
            self._optimize(exchange)
        mark("update")

    def optimizer(self, lr=None, exchange=None):
        if lr is not None:
            self.set_lr(lr)
        self._optimize(exchange)

    def set_lr(self, lr):
        """Device-resident learning rate (train.py:137-142 cosine schedule), read by Adam."""
        self.lr_dev.fill_(float(lr))

    def step(self, batch: Batch):
        self.run(batch)

    # ---------------------------------------------------------------- HIP graphs
    def capture(self, host_noise=False):
        """Capture the step as HIP graphs over two alternating march buffer sets j = 0, 1.

        One part, no collective (the default N=1 step): ONE graph per step ("step": chain -> scatter
        with the whole optimizer in its launches -> repack); the next step's batch draw + march is a
        graph of its own on a side stream, started by a device gate the step graph opens as the
        table-gradient scatter begins (gate.hip).  Data parallel (one part): TWO graphs per step around
        the collective ("dp_pre": repack -> chain -> scatter -> float gradient -> non-finite flag
        into the shards; "dp_post": flag back -> Adam on this rank's shard (sharded) or everywhere
        (all-reduce)), the collectives issued stream-ordered between them, the march gated the same
        way.  The per-stage graphs (march[j], chain[j][q], grid_bw[j][q], finish, update / adam +
        pack) serve several parts and the steps whose scatter is timed by events (bench).
        host_noise: the march perturbation is copied from a buffer replay(noise=...) fills instead of
        drawn from the step's generator (parity tests driving several processes with one draw).
        Call after at least one eager step (lazy library init happens outside capture)."""
        N = self.cfg.n_rays
        self._flush_pack()
        if len(self.mbuf) == 1:
            self.mbuf.append(self._march_buffers())
        self._static = [_packed_batch(torch.zeros(3, N, 3, device=self.dev)) for _ in range(2)]
        self._host_noise = bool(host_noise)
        self._static_noise = [torch.zeros(N, device=self.dev) for _ in range(2)] if host_noise else None
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        nomark = lambda _n: None  # noqa: E731

        def cap(fn, rng=False):
            g = torch.cuda.CUDAGraph()
            if rng:
                g.register_generator_state(self.gen)
            with torch.cuda.graph(g, pool=pool):
                fn()
            return g

        P = self.n_parts
        def march(j):
            if self.dataset is not None:
                self._draw(self._static[j], self.mbuf[j])
            self._march(self._static[j], self.mbuf[j], nomark, prepped=self.dataset is not None,
                        noise=self._static_noise[j] if host_noise else None)

        self.graphs = {
            "march": [cap(lambda j=j: march(j), rng=True) for j in range(2)],
            "chain": [[cap(lambda j=j, q=q: self._chain(self._static[j], self.mbuf[j], q, nomark)) for q in range(P)]
                      for j in range(2)],
            "grid_bw": [[cap(lambda j=j, q=q: self._grid_bw(self.mbuf[j], q)) for q in range(P)] for j in range(2)],
            "finish": [cap(lambda q=q: self._grid_finish(q)) for q in range(P)],
            "reduce": cap(self._reduce_parts) if P > 1 else None,
        }
        # one part: the next step's march waits on the side stream for the gate the step graph opens
        # as its scatter begins (the dense-level launch's first workgroup, or a signal kernel)
        gated = P == 1
        self._gate = torch.zeros(4, dtype=torch.int32, device=self.dev)  # {signals, waits, -, timeouts}
        gp = ptr(self._gate) if gated else None
        self._gate_opened = 0
        if gated:
            self.graphs["march_gated"] = [
                cap(lambda j=j: (call("mfnerf_gate_wait", gp, GATE_TIMEOUT_US, stream()), march(j)), rng=True)
                for j in range(2)]
        amp = self._amp_on()
        self.graphs["pack"] = cap(self._pack)
        if self.shard is not None:
            rank, lo, hi = self.shard
            self.graphs["adam"] = cap(lambda: self._adam(self.g_shard, lo, hi, False))
        else:
            self.graphs["update"] = cap(self._update)
        if P == 1:
            # data parallel: the step up to the exchange, then the update after it
            w = self.shard[2] - self.shard[1] if self.shard is not None else self.n_alloc
            n_sh = self.n_alloc // w
            # sharded with amp: one launch reads the exchanged flag, updates and zeroes level_l1
            fused_shard = amp and self.shard is not None

            def dp_pre(j):
                self._pack()  # the previous step's all-gathered / updated fp16 weights
                self._chain(self._static[j], self.mbuf[j], 0, nomark)
                # the non-finite flag rides the collective: NaN into every shard's first value (by
                # the float finish when it can, else a launch of its own)
                sf = (ptr(self.finite_status), n_sh, w) if amp else None
                folded = self._grid_bw_float(self.mbuf[j], zero_l1=not fused_shard, gate=gp, shard_flag=sf)
                if amp and not folded:
                    call("mfnerf_flag_to_shards", ptr(self.grads), n_sh, w, ptr(self.finite_status), stream())

            def dp_post():
                if fused_shard:
                    self._adam_shard()
                elif self.shard is not None:
                    if amp:
                        call("mfnerf_flag_from_shard", ptr(self.g_shard), ptr(self.finite_status), stream())
                    self._adam(self.g_shard, self.shard[1], self.shard[2], False)
                else:
                    if amp:
                        call("mfnerf_flag_from_shard", ptr(self.grads), ptr(self.finite_status), stream())
                    self._adam(self.grads, 0, self.n_alloc, True)
            self.graphs["dp_pre"] = [cap(lambda j=j: dp_pre(j)) for j in range(2)]
            self.graphs["dp_post"] = cap(dp_post)
            from . import dp as _dp
            if _dp.direct_rccl() is not None:
                # RCCL on this stream (mfnerf.rccl): the collectives are captured too, and the whole
                # data-parallel step (repack, chain, scatter, exchange, Adam, all-gather) replays as
                # ONE graph -- no host hop between the backward and the update
                def dp_step(j):
                    dp_pre(j)
                    if self.shard is not None:
                        _dp.reduce_scatter_mean_(self.g_shard, self.grads)
                        dp_post()
                        _dp.all_gather_(self.p16, self.shard[0])
                    else:
                        _dp.allreduce_mean_(self.grads)
                        dp_post()
                self.graphs["dp_step"] = [cap(lambda j=j: dp_step(j)) for j in range(2)]
        if self.shard is None and P == 1:
            tail = self._finish_update if self._fixed() else lambda: (self._grid_finish(0), self._update())
            self.graphs["finish_update"] = cap(tail)
            fuse = self._fixed() and self._fused_adam_ok()
            # the scatter with the optimizer (one graph transition less) for untimed steps
            if fuse:  # the whole optimizer inside the scatter's launches
                self.graphs["grid_bw_tail"] = [cap(lambda j=j: self._fused_tail(j)) for j in range(2)]
            else:
                self.graphs["grid_bw_tail"] = [cap(lambda j=j: (self._grid_bw(self.mbuf[j], 0), tail()))
                                               for j in range(2)]

            # the whole step as ONE graph: the scatter opens the device gate where the host used to
            # record the event that starts the next march
            def step(j):
                self._chain(self._static[j], self.mbuf[j], 0, nomark)
                if fuse:
                    self._fused_tail(j, gate=gp)
                else:
                    self._grid_bw(self.mbuf[j], 0, gate=gp)
                    tail()
            self.graphs["step"] = [cap(lambda j=j: step(j)) for j in range(2)]
        n_gated = 2 * sum(1 for k in ("step", "dp_pre", "dp_step") if self.graphs.get(k) is not None)
        if gated and self._gate_opened != n_gated:
            # every gated graph must open the gate exactly once, or each gated march would spin for
            # GATE_TIMEOUT_US before starting
            raise RuntimeError(f"gated graphs opened the gate {self._gate_opened} times, not {n_gated}")
        torch.cuda.synchronize()
        # the side stream at normal queue priority: a high-priority one measured the same alone
        # (0.601 vs 0.601 ms/step) but, once an RCCL communicator exists in the process, it ran every
        # step at 1.10 ms (kernels on the main queue 2-7x slower; the extra streams share hardware
        # queues) -- the data-parallel step would pay it on every rank.  No priority below normal
        # exists here (torch.cuda.Stream.priority_range() is (0, -1) on this ROCm, r4m).
        self._side = torch.cuda.Stream(device=self.dev, priority=0)
        self._part_streams = [None] + [torch.cuda.Stream(device=self.dev) for _ in range(P - 1)]
        self._ev_march = [torch.cuda.Event(), torch.cuda.Event()]
        self._ev_start = torch.cuda.Event()
        self._ev_chain = [torch.cuda.Event() for _ in range(P)]
        self._ev_part = [torch.cuda.Event() for _ in range(P)]
        self._parity = 0
        self._primed = False

    def gate_timeouts(self):
        """Gated marches that started on the gate's timeout instead of its signal (gate.hip's gate[3],
        cumulative; a host read, so it synchronises): non-zero means a step paid up to GATE_TIMEOUT_US
        -- e.g. the side stream shares a hardware queue with the stream that signals."""
        g = getattr(self, "_gate", None)
        return 0 if g is None else int(g[3])

    def _fused_tail(self, j, gate=None):
        """The replayed collective-free tail: the scatter with every Adam update in its launches
        (mfnerf_grid_encode_bw_binned_adam_all: the MLPs' and dense levels' update rides the
        accumulate's launch) and the MLP repack; gate: opened as the scatter starts."""
        self._grid_bw(self.mbuf[j], 0, fuse_adam="all", gate=gate)

    def _stage_batch(self, j, batch):
        dst = self._static[j]
        if getattr(batch, "buf", None) is not None:
            dst.buf.copy_(batch.buf)
        else:
            for d, s_ in zip((dst.rays_o, dst.rays_d, dst.rgb), (batch.rays_o, batch.rays_d, batch.rgb)):
                d.copy_(s_)

    def _march_on_side(self, j, batch, after, gated=False, noise=None):
        """Copy batch (and, captured with host_noise, its perturbation) into static set j and march
        it on the side stream once `after` (an event on the main stream) has passed: set j's buffers
        were last read two steps back.  gated: the march graph first waits (a polling wave, at most
        GATE_TIMEOUT_US) for the step graph's gate signal (placement only)."""
        self._side.wait_event(after)
        with torch.cuda.stream(self._side):
            if batch is not None:
                self._stage_batch(j, batch)
            if self._host_noise:
                if noise is None:
                    raise ValueError("captured with host_noise: pass noise= / next_noise= to replay()")
                self._static_noise[j].copy_(noise)
            self.graphs["march_gated" if gated else "march"][j].replay()
            self._ev_march[j].record(self._side)

    def replay(self, batch: Batch = None, exchange=None, grid_bw_events=None, next_batch=None, prefetch=None,
               noise=None, next_noise=None):
        """One training step from the captured graphs (the kernels of run()).  With next_batch (or,
        with an attached dataset, prefetch=True, its default), the next step's march is issued on
        the side stream to overlap this step; the next replay() must then be called with that batch
        (or, with a dataset, the next replay() trains on the batch already drawn).  Pass
        prefetch=False before anything that must precede the next march (an occupancy refresh).
        Data parallel: sharded (shard_optimizer) or exchange=dp.allreduce_mean_.
        grid_bw_events: optional (start, [end per part]) timing events -- start before part 0's
        grid_bw, end after each part's grid_bw (that step runs the per-stage graphs).
        noise / next_noise: the perturbations of batch / next_batch (capture(host_noise=True))."""
        from . import dp
        g, j, P = self.graphs, self._parity, self.n_parts
        dp_mode = self.shard is not None or exchange is not None
        if self.dataset is not None:
            batch = None
            if prefetch is None:
                prefetch = True
        elif prefetch is None:
            prefetch = next_batch is not None
        elif prefetch and next_batch is None:
            raise ValueError("prefetch needs next_batch (or an attached dataset)")
        main = torch.cuda.current_stream()
        self._ev_start.record(main)
        if not self._primed:
            self._march_on_side(j, batch, self._ev_start, noise=noise)
        one_graph = P == 1 and grid_bw_events is None and prefetch and g.get("march_gated") is not None
        if one_graph and (dp_mode or g.get("step") is not None):
            # set 1-j was last read by the previous step, all of which precedes _ev_start
            main.wait_event(self._ev_march[j])
            self._use(self.mbuf[j])
            self.last_batch = self._static[j]
            self.adam_step += 1
            if not dp_mode:  # one graph for the step; the next march starts at its gate signal
                g["step"][j].replay()
                self._march_on_side(1 - j, next_batch, self._ev_start, gated=True, noise=next_noise)
            elif g.get("dp_step") is not None and (self.shard is not None or exchange is dp.allreduce_mean_):
                # the whole data-parallel step, collectives included, as one graph (direct RCCL)
                g["dp_step"][j].replay()
                self._march_on_side(1 - j, next_batch, self._ev_start, gated=True, noise=next_noise)
                self._stale_pack = True  # the next step's graph starts with the repack
            else:
                # [repack] chain, scatter, float gradient, flag -> collective -> Adam -> (all-gather)
                g["dp_pre"][j].replay()
                self._march_on_side(1 - j, next_batch, self._ev_start, gated=True, noise=next_noise)
                if self.shard is not None:
                    dp.reduce_scatter_mean_(self.g_shard, self.grads)
                    g["dp_post"].replay()
                    dp.all_gather_(self.p16, self.shard[0])
                else:
                    exchange(self.grads)
                    g["dp_post"].replay()
                self._stale_pack = True  # the next step's dp_pre (or the pack graph) repacks
            self._parity = 1 - j
            self._primed = True
            return
        fuse_tail = g.get("finish_update") is not None and not dp_mode
        self._flush_pack()
        main.wait_event(self._ev_march[j])
        self._use(self.mbuf[j])
        self.last_batch = self._static[j]
        for q in range(P):
            sq = main if q == 0 else self._part_streams[q]
            if q > 0:
                sq.wait_event(self._ev_chain[q - 1])
            with torch.cuda.stream(sq):
                g["chain"][j][q].replay()
                self._ev_chain[q].record(sq)
                if q == P - 1 and prefetch:
                    # set 1-j was last read by the previous step, which this chain follows; waiting
                    # for the last chain puts the march under the grid_bw scatters, not the chains
                    self._march_on_side(1 - j, next_batch, self._ev_chain[q], noise=next_noise)
                if fuse_tail and grid_bw_events is None:
                    # P == 1: scatter + convert/Adam + repack as one graph (no event needed between)
                    self.adam_step += 1
                    g["grid_bw_tail"][j].replay()
                    self._ev_part[q].record(sq)
                    continue
                if grid_bw_events is not None and q == 0:
                    grid_bw_events[0].record(sq)
                g["grid_bw"][j][q].replay()
                if grid_bw_events is not None:
                    grid_bw_events[1][q].record(sq)
                if q > 0:  # the folds read-modify-write the shared gradient: one part at a time
                    sq.wait_event(self._ev_part[q - 1])
                if not fuse_tail:
                    g["finish"][q].replay()
                self._ev_part[q].record(sq)
        for q in range(1, P):
            main.wait_event(self._ev_part[q])
        if g["reduce"] is not None:
            g["reduce"].replay()
        if self.shard is not None:
            self._optimize(None, adam=lambda _g: self._shard_adam(g["adam"].replay),
                           pack=g["pack"].replay)
        elif fuse_tail and grid_bw_events is None:
            pass  # replayed with the scatter above
        elif fuse_tail:
            self.adam_step += 1
            g["finish_update"].replay()
        else:
            self._optimize(exchange, adam=lambda _g: g["update"].replay())
        self._parity = 1 - j
        self._primed = bool(prefetch)

    # ---------------------------------------------------------------- occupancy (networks.py:157-271)
    def _occ_buffers(self):
        """Scratch for the refresh, sized for the warm-up (all cells) case, allocated once."""
        if getattr(self, "_occ", None) is None:
            lib, c, C, G = load(), self.cfg, self.cascades, self.G
            # one point per distinct drawn cell (mfnerf_occupancy_cells_unique_dev): at most every cell
            n = max(lib.mfnerf_occupancy_points_unique(C, G, G ** 3 // 4, 0), lib.mfnerf_occupancy_points(C, G, 0, 1))
            o = _State()
            o.n_max = n
            o.xyz = torch.empty(n, 3, dtype=torch.float32, device=self.dev)
            o.cell = torch.empty(n, dtype=torch.int32, device=self.dev)
            o.feat = torch.empty(c.L, n, c.F, dtype=torch.float16, device=self.dev)  # level planes
            o.sigma = torch.empty(n, dtype=torch.float32, device=self.dev)
            o.tmp = torch.zeros(C * G ** 3, dtype=torch.float32, device=self.dev)  # kept zero by the decay
            o.ws = torch.zeros(lib.mfnerf_occupancy_workspace(C, G), dtype=torch.uint8, device=self.dev)
            o.count = torch.zeros(1, dtype=torch.int32, device=self.dev)  # probed (distinct) cells
            o.calls = torch.zeros(1, dtype=torch.int64, device=self.dev)  # the draws' call index (device)
            o.graphs = {}
            self._occ = o
        return self._occ

    @torch.no_grad()
    def update_density_grid(self, warmup=False, decay=0.95, count_grid=None, seed=0):
        """NGP.update_density_grid(0.01*MAX_SAMPLES/sqrt(3), warmup, erode) as device launches only
        (cells -> grid_encode_fw -> field_fw density-only + scatter -> decay/mean -> thr + packbits); no
        host synchronisation.  Without erosion (count_grid) the launches are captured once per
        (warmup, decay, seed) and replayed as one HIP graph (the draws' call index lives on the
        device, so every replay draws new cells): 0.45 ms of mostly launch overhead eagerly
        (DESIGN.md 6)."""
        o = self._occ_buffers()
        self._flush_pack()  # the density query runs the field on `packed`
        if count_grid is not None:
            self._occ_launches(warmup, decay, count_grid, seed)
            return
        key = (bool(warmup), float(decay), int(seed))
        g = o.graphs.get(key)
        if g is None:
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._occ_launches(warmup, decay, None, seed)
            o.graphs[key] = g  # (capturing ran nothing)
        g.replay()

    def _occ_launches(self, warmup, decay, count_grid, seed):
        c, C, G, s = self.cfg, self.cascades, self.G, stream()
        o = self._occ_buffers()
        thr = 0.01 * MAX_SAMPLES / SQRT3
        M = G ** 3 // 4
        # the draws of sample_uniform_and_occupied_cells / get_all_cells reduced to one jittered point per
        # distinct drawn cell (the only sigmas the grid can keep), in row-major cell order; count on the device
        n = load().mfnerf_occupancy_points_unique(C, G, M, int(warmup))
        call("mfnerf_occupancy_cells_unique_dev", ptr(self.density_grid), C, G, float(c.scale), M, int(warmup), thr,
             seed, ptr(o.calls), ptr(o.xyz), ptr(o.cell), ptr(o.count), ptr(o.ws), s)
        call("mfnerf_grid_encode_fw_planar", ptr(o.xyz), n, ptr(o.count), self.x_min, self.x_range, self.desc,
             ptr(self.p16[self.off_table:]), ptr(o.feat), o.n_max, s)
        # sigma + density_grid_tmp[cell] = sigma in one launch; the update then starts at the decay
        call("mfnerf_field_fw_density_scatter", ptr(o.feat), o.n_max, n, ptr(o.count), ptr(self.packed), c.rgb_width,
             ptr(o.sigma), ptr(o.cell), ptr(o.tmp), s)
        call("mfnerf_occupancy_update_dev", ptr(self.density_grid), None, None, 0, None, C, G, float(decay),
             ptr(count_grid) if count_grid is not None else None, thr, ptr(o.tmp), 1, ptr(self.bitfield), ptr(o.ws), s)

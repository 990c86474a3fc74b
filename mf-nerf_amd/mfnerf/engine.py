"""The fused MI355X training step: one NeRF training iteration of the reference's hot path
(train.py:164-190 -> rendering.py:121-163 -> losses.py:47-60 -> backward -> FusedAdam) as a
fixed sequence of gfx950 kernels on one stream, with every intermediate resident in HBM and the
sample count kept on the device (no host synchronisation, so a step is capturable in a HIP graph).

Buffers are sized once for the worst case (n_rays * MAX_SAMPLES samples, as the reference's
raymarching_train does); kernels that run per sample read the live count from `counter[0]` and
grid-stride over it.  Parameters live in one flat fp32 vector
    params = [xyz MLP (3072) | rgb MLP (7168) | grid table (L*F*entries)]
so Adam is one launch and the gradient zeroing one memset; an fp16 mirror of the whole vector is
refreshed by the same Adam pass and is what the grid kernels gather from.
Multi-GPU: run(exchange=dp.allreduce_mean_) all-reduces `grads` between the backward and Adam.
"""
import math
from dataclasses import dataclass

import numpy as np
import torch

from . import synthetic
from ._lib import call, load, ptr, stream
from .field import XYZ_NET_PARAMS, rgb_net_params
from .grid import GridLayout

MAX_SAMPLES = 1024
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
    T_threshold: float = 1e-4
    max_samples: int = MAX_SAMPLES


@dataclass
class Batch:
    rays_o: torch.Tensor
    rays_d: torch.Tensor
    rgb: torch.Tensor


class _State:
    pass


def _packed_batch(buf):
    """Batch whose tensors are views into one (3, N, 3) buffer (rays_o, rays_d, rgb)."""
    b = Batch(buf[0], buf[1], buf[2])
    b.buf = buf
    return b


class TrainStep:
    def __init__(self, cfg: StepConfig, device="cuda", seed=0):
        self.cfg = cfg
        self.dev = torch.device(device)
        load()
        c = cfg
        self.cascades = max(1 + int(np.ceil(np.log2(2 * c.scale))), 1)
        self.G = 128
        b = float(np.exp(np.log(c.N_max * c.scale / c.N_min) / (c.L - 1)))
        self.layout = GridLayout(c.L, c.F, c.log2_T, c.N_min, b, c.grid, c.N_tables)
        self.desc = self.layout.desc()
        self.n_rgb = rgb_net_params(c.rgb_width)
        self.off_rgb = XYZ_NET_PARAMS
        self.off_table = XYZ_NET_PARAMS + self.n_rgb
        self.n_params = self.off_table + self.layout.n_params
        s32 = np.float32(c.scale)
        self.x_min, self.x_range = float(-s32), float(np.float32(s32) - np.float32(-s32))

        dev = self.dev
        g = torch.Generator().manual_seed(seed)
        p = torch.empty(self.n_params)
        off = 0
        for o, k in [(64, 32), (16, 64), (c.rgb_width, 32), (c.rgb_width, c.rgb_width), (16, c.rgb_width)]:
            s = math.sqrt(6.0 / (o + k))  # tcnn Xavier-uniform per matrix
            p[off:off + o * k].uniform_(-s, s, generator=g)
            off += o * k
        p[self.off_table:].uniform_(-1e-4, 1e-4, generator=g)  # tcnn grid init
        self.params = p.to(dev)
        self.grads = torch.zeros(self.n_params, device=dev)
        self.m = torch.zeros(self.n_params, device=dev)
        self.v = torch.zeros(self.n_params, device=dev)
        self.p16 = self.params.half()
        self.packed = torch.empty(load().mfnerf_field_packed_bytes(c.rgb_width) // 2, dtype=torch.float16,
                                  device=dev)
        self._pack()
        self.adam_step = 0                                            # host mirror
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)  # Adam's t, bumped on the device
        self.lr_dev = torch.full((1,), float(c.lr), dtype=torch.float32, device=dev)
        self.graphs = None

        # scene bounding box (networks.py:18-23) and occupancy
        self.center = torch.zeros(1, 3, device=dev)
        self.half_size = torch.full((1, 3), c.scale, device=dev)
        self.density_grid = torch.zeros(self.cascades, self.G ** 3, device=dev)
        self.bitfield = torch.zeros(self.cascades * self.G ** 3 // 8, dtype=torch.uint8, device=dev)

        N, cap = c.n_rays, c.n_rays * c.max_samples
        self.cap = cap
        st = _State()
        self.state = st
        f32 = dict(dtype=torch.float32, device=dev)
        self.mbuf = [self._march_buffers()]  # a second set is added by capture() (pipelined march)
        self._use(self.mbuf[0])
        st.feat = torch.empty(cap, c.L * c.F, dtype=torch.float16, device=dev)
        st.sigma = torch.empty(cap, **f32)
        st.rgb_s = torch.empty(cap, 3, **f32)
        st.total = torch.empty(N, dtype=torch.int64, device=dev)
        st.opacity = torch.empty(N, **f32)
        st.depth = torch.empty(N, **f32)
        st.rgb = torch.empty(N, 3, **f32)
        st.ws = torch.empty(cap, **f32)
        st.dL_drgb = torch.empty(N, 3, **f32)
        st.dL_dop = torch.empty(N, **f32)
        st.zeros_ray = torch.zeros(N, **f32)       # dL/ddepth (unused by the loss)
        st.zeros_samp = torch.zeros(cap, **f32)    # dL/dws (no distortion loss by default)
        st.dsig = torch.empty(cap, **f32)
        st.drgb_s = torch.empty(cap, 3, **f32)
        st.dfeat = torch.empty(cap, c.L * c.F, **f32)
        st.field_ws = torch.empty(load().mfnerf_field_bw_workspace(cap, c.rgb_width) // 4, **f32)
        st.loss_sum = torch.zeros(1, **f32)
        st.grid_ws = torch.zeros(max(16, load().mfnerf_grid_encode_bw_workspace(self.desc)) // 4, **f32)
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed + 1)
        # fp16 backward scale: per-sample grads are O(1/n_rays); 2^(floor(log2 N)-2) keeps them normal
        self.grad_scale = float(2.0 ** max(0, int(math.floor(math.log2(N))) - 2))

    MARCH_FIELDS = ("hit_cnt", "hits", "hits_t", "hits_idx", "noise", "rays_a", "xyzs", "dirs", "deltas", "ts",
                    "counter", "march_ws")

    def _march_buffers(self):
        """One set of ray-march outputs (and their scratch), sized for n_rays * MAX_SAMPLES."""
        N, cap, dev = self.cfg.n_rays, self.cap, self.dev
        f32 = dict(dtype=torch.float32, device=dev)
        m = _State()
        m.hit_cnt = torch.empty(N, dtype=torch.int32, device=dev)
        m.hits = torch.empty(N, 1, 2, **f32)
        m.hits_t = m.hits[:, 0]
        m.hits_idx = torch.empty(N, 1, dtype=torch.int64, device=dev)
        m.noise = torch.empty(N, **f32)
        m.rays_a = torch.empty(N, 3, dtype=torch.int64, device=dev)
        m.xyzs = torch.empty(cap, 3, **f32)
        m.dirs = torch.empty(cap, 3, **f32)
        m.deltas = torch.empty(cap, **f32)
        m.ts = torch.empty(cap, **f32)
        m.counter = torch.zeros(2, dtype=torch.int32, device=dev)
        m.march_ws = torch.empty(max(16, load().mfnerf_raymarching_train_workspace(N)), dtype=torch.uint8, device=dev)
        return m

    def _use(self, mb):
        """Point state.<march field> at the buffer set of the step being run (for callers that
        inspect state.rays_a / state.counter / ... after a step)."""
        for k in self.MARCH_FIELDS:
            setattr(self.state, k, getattr(mb, k))

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
        call("mfnerf_field_pack_weights", ptr(self.params), ptr(self.params[self.off_rgb:]), self.cfg.rgb_width,
             ptr(self.packed), stream())

    # ---------------------------------------------------------------- the step
    def _march(self, batch: Batch, mb, mark):
        """Segment 0: AABB + near clamp + noise + ray march into the buffer set mb."""
        c, s = self.cfg, stream()
        N, cap = c.n_rays, self.cap
        # rendering.py:27-29 (AABB + near clamp), custom_functions.py:83 (noise)
        call("mfnerf_ray_aabb_intersect", ptr(batch.rays_o), ptr(batch.rays_d), ptr(self.center),
             ptr(self.half_size), N, 1, 1, ptr(mb.hit_cnt), ptr(mb.hits), ptr(mb.hits_idx), s)
        t1 = mb.hits[:, 0, 0]
        t1.masked_fill_((t1 >= 0) & (t1 < NEAR_DISTANCE), NEAR_DISTANCE)
        torch.rand(N, generator=self.gen, device=self.dev, out=mb.noise)
        mark("prep")
        call("mfnerf_raymarching_train", ptr(batch.rays_o), ptr(batch.rays_d), ptr(mb.hits_t), 2, ptr(self.bitfield),
             self.cascades, float(c.scale), 0.0 if c.scale <= 0.5 else 1 / 256, ptr(mb.noise), self.G,
             c.max_samples, N, cap, ptr(mb.rays_a), ptr(mb.xyzs), ptr(mb.dirs), ptr(mb.deltas), ptr(mb.ts),
             ptr(mb.counter), ptr(mb.march_ws), s)
        mark("march")

    def _fwbw(self, batch: Batch, mb, mark):
        """Segment 1: encode -> field -> composite -> loss -> composite bw -> field bw on mb's samples."""
        c, st, s = self.cfg, self.state, stream()
        N, cap = c.n_rays, self.cap
        call("mfnerf_grid_encode_fw", ptr(mb.xyzs), cap, ptr(mb.counter), self.x_min, self.x_range, self.desc,
             ptr(self.p16[self.off_table:]), ptr(st.feat), s)
        mark("grid_fw")
        call("mfnerf_field_fw", ptr(st.feat), ptr(mb.dirs), cap, ptr(mb.counter), ptr(self.packed), c.rgb_width, 0,
             ptr(st.sigma), ptr(st.rgb_s), s)
        mark("field_fw")
        call("mfnerf_composite_train_fw", ptr(st.sigma), ptr(st.rgb_s), ptr(mb.deltas), ptr(mb.ts), ptr(mb.rays_a),
             N, cap, c.T_threshold, ptr(st.total), ptr(st.opacity), ptr(st.depth), ptr(st.rgb), ptr(st.ws), s)
        bg = 1.0 if c.scale <= 0.5 else 0.0
        st.loss_sum.zero_()
        call("mfnerf_nerf_loss", ptr(st.rgb), ptr(st.opacity), ptr(batch.rgb), N, c.lambda_opacity, bg, bg, bg,
             ptr(st.dL_drgb), ptr(st.dL_dop), ptr(st.loss_sum), s)
        mark("composite_fw")
        call("mfnerf_composite_train_bw", ptr(st.dL_dop), ptr(st.zeros_ray), ptr(st.dL_drgb), ptr(st.zeros_samp),
             ptr(st.sigma), ptr(st.rgb_s), ptr(st.ws), ptr(mb.deltas), ptr(mb.ts), ptr(mb.rays_a), ptr(st.opacity),
             ptr(st.depth), ptr(st.rgb), N, cap, c.T_threshold, ptr(st.dsig), ptr(st.drgb_s), s)
        mark("composite_bw")
        self.grads.zero_()
        call("mfnerf_field_bw", ptr(st.feat), ptr(mb.dirs), cap, ptr(mb.counter), ptr(self.packed), c.rgb_width,
             ptr(st.dsig), ptr(st.drgb_s), self.grad_scale, ptr(st.dfeat), ptr(self.grads),
             ptr(self.grads[self.off_rgb:]), ptr(st.field_ws), s)
        mark("field_bw")

    def _grid_bw(self, mb):
        """Segment 2: the hash-table gradient scatter (the dominant kernel)."""
        st = self.state
        call("mfnerf_grid_encode_bw", ptr(mb.xyzs), self.cap, ptr(mb.counter), self.x_min, self.x_range, self.desc,
             ptr(st.dfeat), ptr(self.grads[self.off_table:]), ptr(st.grid_ws), stream())

    def _update(self):
        """Segment 3: Adam over the flat params (+ fp16 mirror) and the MLP weight repack."""
        c = self.cfg
        call("mfnerf_adam_step", ptr(self.params), ptr(self.grads), ptr(self.m), ptr(self.v), ptr(self.p16),
             self.n_params, float(c.lr), 0.9, 0.999, c.eps, 1.0, 0, ptr(self.step_dev), ptr(self.lr_dev), stream())
        self._pack()

    def run(self, batch: Batch, mark=None, exchange=None):
        """One training step, eagerly, in buffer set 0.  mark(name) is called after each stage
        (bench timing); exchange(grads) runs between backward and Adam (the data-parallel all-reduce)."""
        mark = mark or (lambda name: None)
        mb = self.mbuf[0]
        self._use(mb)
        self._primed = False  # a pipelined replay() must march its own batch next
        self._march(batch, mb, mark)
        self._fwbw(batch, mb, mark)
        self._grid_bw(mb)
        mark("grid_bw")
        if exchange is not None:
            exchange(self.grads)
        mark("allreduce")
        self.optimizer()
        mark("adam")

    def optimizer(self, lr=None):
        if lr is not None:
            self.set_lr(lr)
        self.adam_step += 1
        self._update()

    def set_lr(self, lr):
        """Device-resident learning rate (train.py:137-142 cosine schedule), read by Adam."""
        self.lr_dev.fill_(float(lr))

    def step(self, batch: Batch):
        self.run(batch)

    # ---------------------------------------------------------------- HIP graphs
    def capture(self):
        """Capture the step as HIP graphs over two alternating buffer sets j = 0, 1:
        march[j] (AABB + noise + march of static batch j), fwbw[j], grid_bw[j], and update (Adam +
        repack).  replay() runs march[j'] of the NEXT step on a side stream while grid_bw[j] of this
        one runs on the main stream (the march needs neither this step's gradients nor its update;
        grid_bw is bound by memory-side atomics and leaves the CUs mostly idle).  The split at
        grid_bw also lets the caller time it with events and run the data-parallel all-reduce
        between graphs.  Call after at least one eager step (lazy library init outside capture)."""
        N = self.cfg.n_rays
        if len(self.mbuf) == 1:
            self.mbuf.append(self._march_buffers())
        self._static = [_packed_batch(torch.zeros(3, N, 3, device=self.dev)) for _ in range(2)]
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

        self.graphs = {
            "march": [cap(lambda j=j: self._march(self._static[j], self.mbuf[j], nomark), rng=True) for j in range(2)],
            "fwbw": [cap(lambda j=j: self._fwbw(self._static[j], self.mbuf[j], nomark)) for j in range(2)],
            "grid_bw": [cap(lambda j=j: self._grid_bw(self.mbuf[j])) for j in range(2)],
            "update": cap(self._update),
        }
        torch.cuda.synchronize()
        self._side = torch.cuda.Stream(device=self.dev)
        self._ev_march = [torch.cuda.Event(), torch.cuda.Event()]
        self._ev_fwbw = torch.cuda.Event()
        self._parity = 0
        self._primed = False

    def _stage_batch(self, j, batch):
        dst = self._static[j]
        if getattr(batch, "buf", None) is not None:
            dst.buf.copy_(batch.buf)
        else:
            for d, s_ in zip((dst.rays_o, dst.rays_d, dst.rgb), (batch.rays_o, batch.rays_d, batch.rgb)):
                d.copy_(s_)

    def _march_on_side(self, j, batch):
        """Copy batch into static set j and march it on the side stream (after the main stream's
        work so far: set j's buffers were last read by the grid_bw two steps back)."""
        main = torch.cuda.current_stream()
        self._ev_fwbw.record(main)
        self._side.wait_event(self._ev_fwbw)
        with torch.cuda.stream(self._side):
            self._stage_batch(j, batch)
            self.graphs["march"][j].replay()
            self._ev_march[j].record(self._side)

    def replay(self, batch: Batch, exchange=None, grid_bw_events=None, next_batch=None):
        """One training step from the captured graphs (same kernels as run()).  With next_batch, the
        next step's march is issued on the side stream to overlap this step's grid_bw; the next
        replay() must then be called with that batch.  grid_bw_events: optional (start, end) timing
        events recorded around the grid_bw graph."""
        g, j = self.graphs, self._parity
        main = torch.cuda.current_stream()
        if not self._primed:
            self._march_on_side(j, batch)
        main.wait_event(self._ev_march[j])
        self._use(self.mbuf[j])
        g["fwbw"][j].replay()
        if next_batch is not None:
            self._march_on_side(1 - j, next_batch)
        if grid_bw_events is not None:
            grid_bw_events[0].record(main)
        g["grid_bw"][j].replay()
        if grid_bw_events is not None:
            grid_bw_events[1].record(main)
        if exchange is not None:
            exchange(self.grads)
        self.adam_step += 1
        g["update"].replay()
        self._parity = 1 - j
        self._primed = next_batch is not None

    # ---------------------------------------------------------------- occupancy (networks.py:157-271)
    def _occ_buffers(self):
        """Scratch for the refresh, sized for the warm-up (all cells) case, allocated once."""
        if getattr(self, "_occ", None) is None:
            lib, c, C, G = load(), self.cfg, self.cascades, self.G
            n = max(lib.mfnerf_occupancy_points(C, G, G ** 3 // 4, 0), lib.mfnerf_occupancy_points(C, G, 0, 1))
            o = _State()
            o.n_max = n
            o.xyz = torch.empty(n, 3, dtype=torch.float32, device=self.dev)
            o.cell = torch.empty(n, dtype=torch.int32, device=self.dev)
            o.feat = torch.empty(n, c.L * c.F, dtype=torch.float16, device=self.dev)
            o.sigma = torch.empty(n, dtype=torch.float32, device=self.dev)
            o.tmp = torch.empty(C * G ** 3, dtype=torch.float32, device=self.dev)
            o.ws = torch.empty(lib.mfnerf_occupancy_workspace(C, G), dtype=torch.uint8, device=self.dev)
            o.calls = 0
            self._occ = o
        return self._occ

    @torch.no_grad()
    def update_density_grid(self, warmup=False, decay=0.95, count_grid=None, seed=0):
        """NGP.update_density_grid(0.01*MAX_SAMPLES/sqrt(3), warmup, erode) as five device launches
        (cells -> grid_encode_fw -> field_fw density-only -> scatter/decay/mean -> packbits); no
        host synchronisation, so it can sit inside a captured step sequence."""
        c, C, G, s = self.cfg, self.cascades, self.G, stream()
        o = self._occ_buffers()
        thr = 0.01 * MAX_SAMPLES / SQRT3
        M = G ** 3 // 4
        n = load().mfnerf_occupancy_points(C, G, M, int(warmup))
        call("mfnerf_occupancy_cells", ptr(self.density_grid), C, G, float(c.scale), M, int(warmup), thr, seed,
             o.calls, ptr(o.xyz), ptr(o.cell), ptr(o.ws), s)
        o.calls += 1
        call("mfnerf_grid_encode_fw", ptr(o.xyz), n, None, self.x_min, self.x_range, self.desc,
             ptr(self.p16[self.off_table:]), ptr(o.feat), s)
        call("mfnerf_field_fw", ptr(o.feat), None, n, None, ptr(self.packed), c.rgb_width, 1, ptr(o.sigma), None, s)
        call("mfnerf_occupancy_update", ptr(self.density_grid), ptr(o.sigma), ptr(o.cell), n, C, G, float(decay),
             ptr(count_grid) if count_grid is not None else None, thr, ptr(o.tmp), ptr(self.bitfield), ptr(o.ws), s)

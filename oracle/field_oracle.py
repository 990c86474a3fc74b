"""oracle/field_oracle.py -- TEST INFRASTRUCTURE ONLY (the parity checker).

fp32 torch restatement of the tiny-cuda-nn pieces the reference configures
(models/networks.py:36-79): the multiresolution grid encoding ("HashGrid" and
the MF-NeRF "MixedFeatureGrid"), the degree-4 SphericalHarmonics encoding and
the bias-free FullyFusedMLP.  Differentiable by torch autograd (the grid
backward is torch's index_add scatter).

tiny-cuda-nn is not vendored in the reference, not installed in this image and
its version is unpinned (reference README.md:41, absent from requirements.txt);
the MixedFeature/Window grids and the `n_tables` key come from an unpublished
fork.  PARITY UNPINNED for this file: it restates upstream tcnn's published
HashGrid algorithm (grid.h: grid_scale / grid_resolution / pos_fract /
grid_index / coherent prime hash, table sizing rounded to multiples of 8) and
this repo's documented reading of the MF-NeRF paper (arXiv 2304.12587) for
the mixed-feature table ("MixedFeature").  The HIP kernels are
checked against it to fp16-appropriate tolerances.  The level sizing is
evaluated in fp32 as tcnn does (log2f of the float per_level_scale, exp2f):
at the default Lego config that gives res 65/257/1025 at levels 5/10/15 and
11,445,040 table params (SURVEY.md's 11,420,064 assumed log2 b = 0.4 exactly;
the reference never prints the number, so this stays unpinned too).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes
import ctypes.util
import math

import numpy as np
import torch

_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
for _fn in ("log2f", "exp2f"):
    getattr(_libm, _fn).restype = ctypes.c_float
    getattr(_libm, _fn).argtypes = [ctypes.c_float]


def _f(x):
    return ctypes.c_float(x).value

PRIME1 = 2654435761
PRIME2 = 805459861
GRID_HASH = 0
GRID_MIXED = 1


class GridLayout:
    """Per-level geometry and table offsets (tcnn GridEncodingTemplated constructor sizing)."""

    def __init__(self, n_levels=16, n_features=2, log2_T=19, base_res=16, per_level_scale=1.3195079107728942,
                 grid_type="Hash", n_tables=1):
        self.L, self.F, self.log2_T, self.N_min = n_levels, n_features, log2_T, base_res
        self.b = per_level_scale
        self.grid_type = GRID_MIXED if grid_type in ("MixedFeature", GRID_MIXED) else GRID_HASH
        self.n_tables = max(1, int(n_tables))
        T = 1 << log2_T
        # tcnn evaluates the sizing in fp32: log2f(float(per_level_scale)), exp2f (glibc here)
        log2b = _libm.log2f(_f(per_level_scale))
        self.scales, self.res, self.sizes, self.offsets = [], [], [], []
        self.table_of_level = []  # MixedFeature: shared-table id, -1 for a level-owned table
        off = 0
        for l in range(n_levels):
            # grid_scale: exp2f(level * log2_per_level_scale) * base_resolution - 1.0f
            s = _f(_f(_libm.exp2f(_f(_f(float(l)) * log2b)) * _f(float(base_res))) - 1.0)
            r = int(math.ceil(s)) + 1
            self.scales.append(s)
            self.res.append(r)
        self.dense_levels = [l for l in range(n_levels) if self.res[l] ** 3 <= T]
        hashed = [l for l in range(n_levels) if self.res[l] ** 3 > T]
        for l in range(n_levels):
            if self.grid_type == GRID_MIXED and l in hashed:
                self.sizes.append(0)
                self.offsets.append(-1)
                self.table_of_level.append(hashed.index(l) % self.n_tables)
                continue
            p = self.res[l] ** 3
            p = min(p, 0x7FFFFFFF)
            p = (p + 7) // 8 * 8
            p = min(p, T)
            self.sizes.append(p)
            self.offsets.append(off)
            self.table_of_level.append(-1)
            off += p
        # MixedFeature: n_tables shared tables that together hold 2^log2_T entries
        self.shared_size = 0
        self.shared_offset = off
        if self.grid_type == GRID_MIXED and hashed:
            self.shared_size = max(8, (T // self.n_tables) // 8 * 8)
            for l in range(n_levels):
                if self.table_of_level[l] >= 0:
                    self.offsets[l] = off + self.table_of_level[l] * self.shared_size
                    self.sizes[l] = self.shared_size
            off += self.shared_size * self.n_tables
        self.n_entries = off
        self.n_params = off * n_features
        self.canon_res = self.res[-1]

    def level_arrays(self):
        return (np.array(self.scales, np.float32), np.array(self.res, np.uint32),
                np.array(self.offsets, np.int64), np.array(self.sizes, np.uint32))


def _u32(x):
    return x & 0xFFFFFFFF


def grid_index(layout, l, gx, gy, gz):
    """tcnn grid_index: dense strides while they fit, else the coherent prime hash; `% size`.
    MixedFeature hashed levels first map level coords onto the canonical (finest) grid."""
    size = layout.sizes[l]
    res = layout.res[l]
    if layout.table_of_level[l] >= 0:
        rc = layout.canon_res
        cx, cy, cz = (gx * rc) // res, (gy * rc) // res, (gz * rc) // res
        h = _u32(cx * 1) ^ _u32(cy * PRIME1) ^ _u32(cz * PRIME2)
        return h % size
    stride = 1
    index = torch.zeros_like(gx)
    for g in (gx, gy, gz):
        if stride > size:
            break
        index = index + g * stride
        stride *= res
    if size < stride:
        index = _u32(gx * 1) ^ _u32(gy * PRIME1) ^ _u32(gz * PRIME2)
    return index % size


def _corners(x, layout):
    """Per (level, corner): (flat table row index (N,) i64, trilinear weight (N,) f32)."""
    out = []
    for l in range(layout.L):
        # fmaf(scale, x, 0.5) in fp32: evaluate in fp64 and round once
        pos = (x.double() * float(layout.scales[l]) + 0.5).float()
        g = torch.floor(pos)
        w = pos - g
        gi = g.to(torch.int64)
        lv = []
        for c in range(8):
            gc = [gi[:, d] + ((c >> d) & 1) for d in range(3)]
            wt = torch.ones(x.shape[0], dtype=torch.float32, device=x.device)
            for d in range(3):
                wt = wt * (w[:, d] if (c >> d) & 1 else (1 - w[:, d]))
            lv.append((grid_index(layout, l, gc[0], gc[1], gc[2]) + layout.offsets[l], wt))
        out.append(lv)
    return out


class _GridEncode(torch.autograd.Function):
    """The encoding with the table gradient scattered into ONE buffer (index_add_ per level and
    corner).  Autograd through `table[idx]` would materialise a zero table-sized gradient for each of
    the L*8 gathers (128 x 45 MB per backward at the Lego layout) and sum them."""

    @staticmethod
    def forward(ctx, params, x, layout):
        F = layout.F
        table = params.view(-1, F)
        cs = _corners(x, layout)
        outs = []
        for lv in cs:
            acc = torch.zeros(x.shape[0], F, dtype=torch.float32, device=x.device)
            for idx, wt in lv:
                acc = acc + wt[:, None] * table[idx]
            outs.append(acc)
        ctx.cs, ctx.F, ctx.n, ctx.dtype = cs, F, params.numel(), params.dtype
        return torch.cat(outs, 1)

    @staticmethod
    def backward(ctx, dout):
        F = ctx.F
        grad = torch.zeros(ctx.n // F, F, dtype=ctx.dtype, device=dout.device)
        for l, lv in enumerate(ctx.cs):
            dl = dout[:, l * F:(l + 1) * F]
            for idx, wt in lv:
                grad.index_add_(0, idx, (wt[:, None] * dl).to(ctx.dtype))
        return grad.view(-1), None, None


def grid_encode(x, params, layout):
    """x: (N,3) fp32 in [0,1]; params: (n_params,) fp32 table -> (N, L*F) fp32.
    Per level: pos = fmaf(scale, x, 0.5); g = floor(pos); w = pos - g (Linear);
    out = sum over the 8 corners of prod_d (bit_d ? w_d : 1-w_d) * table[index].
    Differentiable in params (not in x: the encoding's input needs no gradient here)."""
    return _GridEncode.apply(params, x.detach(), layout)


def sh4(d01):
    """tcnn SphericalHarmonics degree 4 on inputs in [0,1]^3 (mapped to [-1,1])."""
    x, y, z = (d01 * 2 - 1).unbind(-1)
    xy, xz, yz, x2, y2, z2 = x * y, x * z, y * z, x * x, y * y, z * z
    out = [
        torch.full_like(x, 0.28209479177387814),
        -0.48860251190291987 * y,
        0.48860251190291987 * z,
        -0.48860251190291987 * x,
        1.0925484305920792 * xy,
        -1.0925484305920792 * yz,
        0.94617469575755997 * z2 - 0.31539156525251999,
        -1.0925484305920792 * xz,
        0.54627421529603959 * x2 - 0.54627421529603959 * y2,
        0.59004358992664352 * y * (-3.0 * x2 + y2),
        2.8906114426405538 * xy * z,
        0.45704579946446572 * y * (1.0 - 5.0 * z2),
        0.3731763325901154 * z * (5.0 * z2 - 3.0),
        0.45704579946446572 * x * (1.0 - 5.0 * z2),
        1.4453057213202769 * z * (x2 - y2),
        0.59004358992664352 * x * (-x2 + 3.0 * y2),
    ]
    return torch.stack(out, -1)


def pad16(n):
    return (n + 15) // 16 * 16


def mlp_shapes(n_in, n_out, n_neurons, n_hidden_layers):
    """FullyFusedMLP weight shapes (out, in), bias-free; the output width is padded to 16."""
    shapes = [(n_neurons, n_in)]
    for _ in range(n_hidden_layers - 1):
        shapes.append((n_neurons, n_neurons))
    shapes.append((pad16(n_out), n_neurons))
    return shapes


def mlp_n_params(n_in, n_out, n_neurons, n_hidden_layers):
    return sum(a * b for a, b in mlp_shapes(n_in, n_out, n_neurons, n_hidden_layers))


def _act(x, name):
    if name in (None, "None"):
        return x
    if name == "ReLU":
        return torch.relu(x)
    if name == "Sigmoid":
        return torch.sigmoid(x)
    if name == "Exponential":
        return torch.exp(x)
    raise ValueError(name)


def mlp_forward(x, params, n_in, n_out, n_neurons, n_hidden_layers, activation="ReLU", output_activation="None"):
    """Row-major W_k (out_k, in_k) blocks concatenated in layer order; returns (N, n_out) fp32."""
    h = x
    off = 0
    shapes = mlp_shapes(n_in, n_out, n_neurons, n_hidden_layers)
    for i, (o, k) in enumerate(shapes):
        W = params[off:off + o * k].view(o, k)
        off += o * k
        h = h @ W.t()
        h = _act(h, activation if i < len(shapes) - 1 else output_activation)
    return h[:, :n_out]


def xavier_uniform_(params, shapes, gen=None):
    off = 0
    with torch.no_grad():
        for o, k in shapes:
            s = math.sqrt(6.0 / (o + k))
            params[off:off + o * k].uniform_(-s, s, generator=gen)
            off += o * k
    return params


# ---- tinycudann-compatible modules (fp32, CPU) used to stub `tinycudann` in fixture generation


class Encoding(torch.nn.Module):
    def __init__(self, n_input_dims, encoding_config, seed=1337, dtype=None):
        super().__init__()
        self.cfg = dict(encoding_config)
        ot = self.cfg.get("otype", "")
        self.kind = "sh" if "SphericalHarmonics" in ot else "grid"
        if self.kind == "sh":
            self.n_output_dims = self.cfg.get("degree", 4) ** 2
            self.params = torch.nn.Parameter(torch.zeros(0))
        else:
            self.layout = layout_from_config(self.cfg)
            self.n_output_dims = self.layout.L * self.layout.F
            g = torch.Generator().manual_seed(seed)
            p = torch.empty(self.layout.n_params).uniform_(-1e-4, 1e-4, generator=g)
            self.params = torch.nn.Parameter(p)

    def forward(self, x):
        if self.kind == "sh":
            return sh4(x.float())
        return grid_encode(x.float(), self.params, self.layout)


def layout_from_config(cfg):
    grid = cfg.get("type", "Hash")
    return GridLayout(cfg["n_levels"], cfg["n_features_per_level"], cfg["log2_hashmap_size"],
                      cfg["base_resolution"], cfg["per_level_scale"], grid, cfg.get("n_tables", 1))


class Network(torch.nn.Module):
    def __init__(self, n_input_dims, n_output_dims, network_config, seed=1337):
        super().__init__()
        c = network_config
        self.n_in, self.n_out = n_input_dims, n_output_dims
        self.width, self.depth = c["n_neurons"], c["n_hidden_layers"]
        self.act, self.out_act = c.get("activation", "ReLU"), c.get("output_activation", "None")
        shapes = mlp_shapes(self.n_in, self.n_out, self.width, self.depth)
        g = torch.Generator().manual_seed(seed)
        self.params = torch.nn.Parameter(xavier_uniform_(torch.empty(sum(a * b for a, b in shapes)), shapes, g))

    def forward(self, x):
        return mlp_forward(x.float(), self.params, self.n_in, self.n_out, self.width, self.depth,
                           self.act, self.out_act)


class NetworkWithInputEncoding(torch.nn.Module):
    """params = [network params | encoding params] (tcnn NetworkWithInputEncoding order)."""

    def __init__(self, n_input_dims, n_output_dims, encoding_config, network_config, seed=1337):
        super().__init__()
        self.enc = Encoding(n_input_dims, encoding_config, seed=seed)
        self.net = Network(self.enc.n_output_dims, n_output_dims, network_config, seed=seed)
        self.n_net = self.net.params.numel()
        self.params = torch.nn.Parameter(torch.cat([self.net.params.data, self.enc.params.data]))
        del self.enc._parameters["params"]
        del self.net._parameters["params"]

    def forward(self, x):
        feat = grid_encode(x.float(), self.params[self.n_net:], self.enc.layout)
        c = self.net
        return mlp_forward(feat, self.params[:self.n_net], c.n_in, c.n_out, c.width, c.depth, c.act, c.out_act)


# ---- fp16-point emulation of the NGP field head (the arithmetic tcnn and the HIP kernels share)


def _h(t):
    return t.half().float()


def ngp_field_fw16(feat16, dirs, px, pr, width=64):
    """NGP.forward's MLP part (networks.py:106,144-147) with every operand rounded to fp16 where
    tcnn holds it in fp16: feat, weights, ReLU outputs, h (the xyz net's half output) and SH.
    Returns sigma (N), rgb (N,3) fp32 and the rounded activations for the backward."""
    f = feat16.float()
    W1 = _h(px[:2048].view(64, 32)); W2 = _h(px[2048:3072].view(16, 64))
    R1 = _h(pr[:width * 32].view(width, 32))
    R2 = _h(pr[width * 32:width * 32 + width * width].view(width, width))
    R3 = _h(pr[width * 32 + width * width:].view(16, width))
    y1 = _h(torch.relu(f @ W1.t()))
    h = _h(y1 @ W2.t())
    dn = dirs / torch.norm(dirs, dim=1, keepdim=True)
    sh = _h(sh4((dn + 1) / 2))
    inp = torch.cat([sh, h], 1)
    r1 = _h(torch.relu(inp @ R1.t()))
    r2 = _h(torch.relu(r1 @ R2.t()))
    rgb = torch.sigmoid((r2 @ R3.t())[:, :3])
    acts = dict(f=f, W1=W1, W2=W2, R1=R1, R2=R2, R3=R3, y1=y1, h=h, inp=inp, r1=r1, r2=r2, rgb=rgb)
    return torch.exp(h[:, 0]), rgb, acts


def ngp_field_bw16(acts, dL_dsigma, dL_drgb, S):
    """Manual backward of ngp_field_fw16 with the incoming grads scaled by S and every data
    gradient rounded to fp16 after its ReLU mask (the fp16 backward products).  Returns
    dL/dfeat (N,32), d xyz-MLP params (3072), d rgb-MLP params, all unscaled fp32."""
    a = acts
    N = a["f"].shape[0]
    rgb = a["rgb"]
    dO = torch.zeros(N, 16)
    dO[:, :3] = dL_drgb * S * rgb * (1 - rgb)
    dO = _h(dO)
    dWr3 = dO.t() @ a["r2"]
    dr2 = _h((dO @ a["R3"]) * (a["r2"] > 0))
    dWr2 = dr2.t() @ a["r1"]
    dr1 = _h((dr2 @ a["R2"]) * (a["r1"] > 0))
    dWr1 = dr1.t() @ a["inp"]
    dh = (dr1 @ a["R1"])[:, 16:].clone()
    dh[:, 0] += dL_dsigma * S * torch.exp(a["h"][:, 0].clamp(-15, 15))  # TruncExp bw
    dh = _h(dh)
    dW2 = dh.t() @ a["y1"]
    dy1 = _h((dh @ a["W2"]) * (a["y1"] > 0))
    dW1 = dy1.t() @ a["f"]
    dX = dy1 @ a["W1"]
    return (dX / S, torch.cat([dW1.flatten(), dW2.flatten()]) / S,
            torch.cat([dWr1.flatten(), dWr2.flatten(), dWr3.flatten()]) / S)

"""tinycudann-compatible modules (the subset MF-NeRF configures, models/networks.py:36-79).

Each module owns one flat fp32 `params` Parameter in tcnn's layout (state-dict keys
`xyz_encoder.params`, `rgb_net.params` as in the reference), initialised like tcnn (grid
U(-1e-4, 1e-4), MLP Xavier-uniform).  NGP (mfnerf.networks) does not call these forwards: it
runs the fused gfx950 field kernels on the same parameters.  The standalone forwards are what the
reference's own networks.py runs with `sys.modules["tinycudann"] = mfnerf.tcnn`:
grids run the HIP grid kernels, the networks the MFMA FullyFusedMLP kernels of mlp.hip
(mfnerf_mlp_fw / _bw), with tcnn's torch-binding loss scale (128) around the fp16 backward.
There is no CPU path: a module on a CPU tensor raises.
"""
import math
import weakref

import torch

from ._lib import call, load, ptr, stream
from .field import GridEncodeFunction
from .grid import GridLayout

# tcnn's torch binding scales the incoming gradient by 128 before its fp16 backward (half params)
# and divides the results by it (tinycudann/modules.py: loss_scale = 128 for fp16 networks)
MLP_LOSS_SCALE = 128.0


def _pad16(n):
    return (n + 15) // 16 * 16


def mlp_shapes(n_in, n_out, n_neurons, n_hidden_layers):
    """FullyFusedMLP weights, bias-free, output width padded to 16: [(out, in), ...]."""
    shapes = [(n_neurons, n_in)] + [(n_neurons, n_neurons)] * (n_hidden_layers - 1)
    return shapes + [(_pad16(n_out), n_neurons)]


def _xavier(shapes, gen):
    parts = []
    for o, k in shapes:
        s = math.sqrt(6.0 / (o + k))
        parts.append(torch.empty(o * k).uniform_(-s, s, generator=gen))
    return torch.cat(parts)


def _act(x, name):
    return {"None": lambda v: v, "ReLU": torch.relu, "Sigmoid": torch.sigmoid, "Exponential": torch.exp}[name](x)


_packed = {}


def _mlp_packed(params, cfg):
    """The MFMA fragment blob of `params` (re-packed only when the parameter changed).  Keyed on
    the storage's owner tensor itself (weakly held), its data pointer and version counter: a new
    tensor that reuses a freed one's memory (and version count) must not hit the old blob."""
    base = params._base if params._base is not None else params
    key = (params.data_ptr(), params.numel(), cfg)
    hit = _packed.get(key)
    if hit is not None and hit[2]() is base and hit[0] == params._version:
        return hit[1]
    n_in, width, depth, n_out = cfg
    nb = load().mfnerf_mlp_packed_bytes(n_in, width, depth, n_out)
    blob = torch.empty(nb // 2, dtype=torch.float16, device=params.device)
    call("mfnerf_mlp_pack", ptr(params.detach().float().contiguous()), n_in, width, depth, n_out, ptr(blob), stream())
    if len(_packed) > 8:
        _packed.clear()
    _packed[key] = (params._version, blob, weakref.ref(base))
    return blob


class MLPFunction(torch.autograd.Function):
    """tcnn FullyFusedMLP forward/backward on the MFMA kernels: x (n, 32) -> (n, n_out) f16."""

    @staticmethod
    def forward(ctx, x, params, cfg, sigmoid):
        if not x.is_cuda:
            raise RuntimeError("mfnerf.tcnn: the networks run on the GPU only (HIP kernels; no CPU path)")
        n_in, width, depth, n_out = cfg
        x16 = x.detach().half().contiguous()
        n = x16.shape[0]
        out = torch.empty(n, 16, dtype=torch.float16, device=x.device)
        call("mfnerf_mlp_fw", ptr(x16), n, ptr(_mlp_packed(params, cfg)), n_in, width, depth, n_out, int(sigmoid),
             ptr(out), stream())
        ctx.save_for_backward(x16, params)
        ctx.cfg, ctx.sigmoid, ctx.x_dtype = cfg, sigmoid, x.dtype
        return out[:, :n_out]

    @staticmethod
    def backward(ctx, dout):
        x16, params = ctx.saved_tensors
        n_in, width, depth, n_out = ctx.cfg
        n = x16.shape[0]
        d16 = torch.zeros(n, 16, dtype=torch.float16, device=x16.device)
        d16[:, :n_out] = (dout.float() * MLP_LOSS_SCALE).half()
        dx = torch.empty(n, n_in, dtype=torch.float32, device=x16.device)
        g = torch.zeros(params.numel(), dtype=torch.float32, device=x16.device)
        ws = torch.empty(max(16, load().mfnerf_mlp_bw_workspace(n, n_in, width, depth, n_out)), dtype=torch.uint8,
                         device=x16.device)
        call("mfnerf_mlp_bw", ptr(x16), n, ptr(_mlp_packed(params, ctx.cfg)), n_in, width, depth, n_out,
             int(ctx.sigmoid), ptr(d16), ptr(dx), ptr(g), ptr(ws), stream())
        dx.mul_(1.0 / MLP_LOSS_SCALE)
        g.mul_(1.0 / MLP_LOSS_SCALE)
        return dx.to(ctx.x_dtype), g.to(params.dtype), None, None


def mlp_forward(x, params, width, depth, n_out, activation, output_activation):
    if activation != "ReLU" or output_activation not in ("None", "Sigmoid") or x.shape[1] != 32:
        raise NotImplementedError(f"FullyFusedMLP({x.shape[1]} in, {activation}/{output_activation}) is outside "
                                  "MF-NeRF's configuration")
    return MLPFunction.apply(x, params, (32, int(width), int(depth), int(n_out)), output_activation == "Sigmoid")


def mlp_forward_fp16(x, params, shapes, n_out, activation, output_activation):
    """The same network as a torch fp16 GEMM chain (test reference for the MFMA kernels)."""
    h = x.half()
    off = 0
    for i, (o, k) in enumerate(shapes):
        W = params[off:off + o * k].view(o, k).half()
        off += o * k
        h = _act(h @ W.t(), activation if i < len(shapes) - 1 else output_activation)
    return h[:, :n_out]


class Encoding(torch.nn.Module):
    """tcnn.Encoding for {Hash,MixedFeature}Grid and SphericalHarmonics (degree 4)."""

    def __init__(self, n_input_dims, encoding_config, seed=1337, dtype=None):
        super().__init__()
        self.n_input_dims = n_input_dims
        self.encoding_config = dict(encoding_config)
        otype = self.encoding_config.get("otype", "")
        if "SphericalHarmonics" in otype:
            self.kind = "sh"
            self.n_output_dims = self.encoding_config.get("degree", 4) ** 2
            self.params = torch.nn.Parameter(torch.zeros(0))
        elif otype.endswith("Grid"):
            self.kind = "grid"
            self.layout = GridLayout.from_config(self.encoding_config)
            self.desc = self.layout.desc()
            self.n_output_dims = self.layout.L * self.layout.F
            g = torch.Generator().manual_seed(seed)
            self.params = torch.nn.Parameter(torch.empty(self.layout.n_params).uniform_(-1e-4, 1e-4, generator=g))
        else:
            raise NotImplementedError(f"encoding {otype} is outside MF-NeRF's configuration")

    def forward(self, x):
        if self.kind == "grid":
            return GridEncodeFunction.apply(x, self.params, self.layout, self.desc)
        if x.is_cuda and not (torch.is_grad_enabled() and x.requires_grad) and self.n_output_dims == 16:
            return sh4_fw(x)  # the HIP kernel (the reference feeds it rays, which carry no gradient)
        return sh4_torch(x.float()).half()


def sh4_fw(d01):
    """(n, 3) directions mapped to [0, 1] -> (n, 16) f16 SH degree 4 (mfnerf_sh4_fw; the same IEEE
    operations as sh4_torch)."""
    lead = d01.shape[:-1]
    x = d01.reshape(-1, 3).float().contiguous()
    out = torch.empty(x.shape[0], 16, dtype=torch.float16, device=x.device)
    call("mfnerf_sh4_fw", ptr(x), x.shape[0], ptr(out), stream())
    return out.reshape(*lead, 16)


def sh4_torch(d01):
    x, y, z = (d01 * 2 - 1).unbind(-1)
    xy, xz, yz, x2, y2, z2 = x * y, x * z, y * z, x * x, y * y, z * z
    return torch.stack([
        torch.full_like(x, 0.28209479177387814), -0.48860251190291987 * y, 0.48860251190291987 * z,
        -0.48860251190291987 * x, 1.0925484305920792 * xy, -1.0925484305920792 * yz,
        0.94617469575755997 * z2 - 0.31539156525251999, -1.0925484305920792 * xz,
        0.54627421529603959 * x2 - 0.54627421529603959 * y2, 0.59004358992664352 * y * (-3.0 * x2 + y2),
        2.8906114426405538 * xy * z, 0.45704579946446572 * y * (1.0 - 5.0 * z2),
        0.3731763325901154 * z * (5.0 * z2 - 3.0), 0.45704579946446572 * x * (1.0 - 5.0 * z2),
        1.4453057213202769 * z * (x2 - y2), 0.59004358992664352 * x * (-x2 + 3.0 * y2)], -1)


class Network(torch.nn.Module):
    """tcnn.Network with a FullyFusedMLP config."""

    def __init__(self, n_input_dims, n_output_dims, network_config, seed=1337):
        super().__init__()
        c = network_config
        self.n_input_dims, self.n_output_dims = n_input_dims, n_output_dims
        self.width, self.depth = c["n_neurons"], c["n_hidden_layers"]
        self.activation, self.output_activation = c.get("activation", "ReLU"), c.get("output_activation", "None")
        self.shapes = mlp_shapes(n_input_dims, n_output_dims, self.width, self.depth)
        g = torch.Generator().manual_seed(seed)
        self.params = torch.nn.Parameter(_xavier(self.shapes, g))

    def forward(self, x):
        return mlp_forward(x, self.params, self.width, self.depth, self.n_output_dims, self.activation,
                           self.output_activation)


class NetworkWithInputEncoding(torch.nn.Module):
    """tcnn.NetworkWithInputEncoding: params = [network (MLP) | encoding (grid)]."""

    def __init__(self, n_input_dims, n_output_dims, encoding_config, network_config, seed=1337):
        super().__init__()
        enc = Encoding(n_input_dims, encoding_config, seed=seed)
        net = Network(enc.n_output_dims, n_output_dims, network_config, seed=seed)
        self.layout, self.desc = enc.layout, enc.desc
        self.n_output_dims = n_output_dims
        self.shapes, self.n_net = net.shapes, net.params.numel()
        self.activation, self.output_activation = net.activation, net.output_activation
        self.width, self.depth = net.width, net.depth
        self.params = torch.nn.Parameter(torch.cat([net.params.data, enc.params.data]))

    def forward(self, x):
        feat = GridEncodeFunction.apply(x, self.params[self.n_net:], self.layout, self.desc)
        return mlp_forward(feat, self.params[:self.n_net], self.width, self.depth, self.n_output_dims,
                           self.activation, self.output_activation)

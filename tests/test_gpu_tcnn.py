"""The tinycudann module route on the MFMA kernels (mlp.hip): mfnerf.tcnn.Network /
NetworkWithInputEncoding as the reference's models/networks.py:36-79 builds them one module at a
time (what runs with sys.modules["tinycudann"] = mfnerf.tcnn).

* the FullyFusedMLP kernels against an fp16-point restatement of tcnn's network (operands rounded
  to fp16 where tcnn rounds them, fp64 sums), forward and backward (torch autograd of the same
  restatement), for every (width, hidden layers, output activation) MF-NeRF configures;
* the three modules composed exactly as networks.py:134-155 (xyz_encoder -> TruncExp(h[:, 0]),
  SH4((d/|d| + 1)/2), rgb_net(cat[SH, h])) against the fused field head (mfnerf.networks.NGP,
  field.hip) on the same parameters: sigma, rgb and the parameter gradients."""
import math

import pytest
import torch

from mfnerf import tcnn
from oracle import field_oracle as FO

pytestmark = pytest.mark.gpu

LEGO_B = math.exp(math.log(2048 * 0.5 / 16) / 15)


def _h(t):
    return t.half().double()


def mlp16(x, params, shapes, n_out, out_act):
    """tcnn FullyFusedMLP in fp16-point arithmetic: each layer's input rounded to fp16, exact sums,
    ReLU'd hidden outputs rounded to fp16, the output activation on the fp16 logits -> fp16."""
    h = _h(x)
    off = 0
    for i, (o, k) in enumerate(shapes):
        W = _h(params[off:off + o * k].view(o, k))
        off += o * k
        z = h @ W.t()
        if i < len(shapes) - 1:
            h = _h(torch.relu(z))
        else:
            h = torch.sigmoid(z) if out_act == "Sigmoid" else z
    return h[:, :n_out]


CFGS = [(64, 1, 16, "None"), (64, 2, 3, "Sigmoid"), (128, 2, 3, "Sigmoid"), (128, 1, 16, "None")]


@pytest.mark.parametrize("width,depth,n_out,out_act", CFGS)
def test_fully_fused_mlp_vs_fp16_oracle(gpu, width, depth, n_out, out_act):
    g = torch.Generator().manual_seed(width + 7 * depth + n_out)
    net = tcnn.Network(32, n_out, {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": out_act,
                                   "n_neurons": width, "n_hidden_layers": depth}, seed=3).to(gpu)
    with torch.no_grad():
        net.params.mul_(2.0)
    n = 1000  # not a multiple of the 32-sample tile
    x = (torch.rand(n, 32, generator=g) * 2 - 1).half()
    dout = torch.randn(n, n_out, generator=g) * 1e-2
    xg = x.to(gpu).requires_grad_(True)
    y = net(xg)
    assert y.dtype == torch.float16 and y.shape == (n, n_out)
    p64 = net.params.detach().cpu().double().requires_grad_(True)
    x64 = x.double().requires_grad_(True)
    ref = mlp16(x64, p64, tcnn.mlp_shapes(32, n_out, width, depth), n_out, out_act)
    # fp32 accumulation of fp16 products vs exact sums, then one fp16 rounding: <= ~2 fp16 ulps
    err = (y.detach().cpu().double() - ref.detach()).abs()
    assert float(err.max()) <= 2e-3 * max(1.0, float(ref.detach().abs().max())), float(err.max())
    (y.float() * dout.to(gpu)).sum().backward()
    (ref * dout.double()).sum().backward()
    # backward: fp16 operands (the loss-scaled dL/dout, activations, weights) with fp32 sums
    gx, gp = xg.grad.double().cpu(), net.params.grad.double().cpu()
    rx = x64.grad
    assert float((gx - rx).norm()) <= 1e-2 * float(rx.norm())
    off = 0
    for o, k in tcnn.mlp_shapes(32, n_out, width, depth):
        a, b = gp[off:off + o * k], p64.grad[off:off + o * k]
        off += o * k
        if float(b.norm()) > 0:  # per layer: a sign error in one block cannot hide in the total
            assert float((a - b).norm()) <= 1e-2 * float(b.norm()), (o, k)
    # deterministic: the weight gradient is summed over sample chunks in a fixed order
    net.params.grad = None
    xg.grad = None
    (net(xg).float() * dout.to(gpu)).sum().backward()
    assert torch.equal(net.params.grad.double().cpu(), gp)


def test_module_route_matches_fused_field(gpu):
    """networks.py:134-155 composed from the standalone modules == the fused field head."""
    from mfnerf.custom_functions import TruncExp
    from mfnerf.networks import NGP

    class HP:
        grid, L, F, T, N_min, N_max, N_tables, rgb_channels, rgb_layers = "Hash", 16, 2, 14, 16, 2048, 1, 64, 2

    model = NGP(scale=0.5, hparams=HP).to(gpu)
    g = torch.Generator().manual_seed(11)
    with torch.no_grad():
        n_net = model.xyz_encoder.n_net
        model.xyz_encoder.params[n_net:].copy_((torch.rand(model.xyz_encoder.params.numel() - n_net,
                                                            generator=g) - 0.5).to(gpu))
        model.xyz_encoder.params[:n_net].mul_(3)
        model.rgb_net.params.mul_(3)
    n = 3000
    x = ((torch.rand(n, 3, generator=g) - 0.5) * 0.98).to(gpu)
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g), dim=-1).to(gpu)
    dsig = (torch.randn(n, generator=g) * 1e-3).to(gpu)
    drgb = (torch.randn(n, 3, generator=g) * 1e-2).to(gpu)
    # the fused head
    sig_f, rgb_f = model(x, d)
    (sig_f * dsig).sum().add_((rgb_f * drgb).sum()).backward()
    gx_f, gr_f = model.xyz_encoder.params.grad.clone(), model.rgb_net.params.grad.clone()
    model.zero_grad()
    # the module route, as networks.py writes it
    xn = (x - model.xyz_min) / (model.xyz_max - model.xyz_min)
    h = model.xyz_encoder(xn)
    sig_m = TruncExp.apply(h[:, 0])
    dn = d / torch.norm(d, dim=1, keepdim=True)
    dd = model.dir_encoder((dn + 1) / 2)
    rgb_m = model.rgb_net(torch.cat([dd, h], 1))
    (sig_m.float() * dsig).sum().add_((rgb_m.float() * drgb).sum()).backward()
    gx_m, gr_m = model.xyz_encoder.params.grad, model.rgb_net.params.grad
    # both are fp16 networks; they differ in where fp16 rounding happens (h feeds the rgb net as
    # fp16 in both) -- outputs to fp16 resolution
    assert torch.allclose(rgb_m.float(), rgb_f, atol=4e-3)
    assert torch.allclose(sig_m.float(), sig_f, rtol=8e-3, atol=1e-5)
    for (a, b) in ((gx_m[:n_net], gx_f[:n_net]), (gx_m[n_net:], gx_f[n_net:]), (gr_m, gr_f)):
        assert float((a - b).norm()) <= 3e-2 * float(b.norm())
        assert float(torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0)) > 0.999


def test_sh4_fw_kernel_matches_the_oracle(gpu):
    """mfnerf_sh4_fw (the tinycudann route's SphericalHarmonics degree 4, networks.py:60-67) against
    the CPU oracle's sh4 (oracle/field_oracle.py, tcnn's published SH basis, one fp32 operation at a
    time, rounded to fp16 once), bit for bit, on directions mapped to [0, 1] as networks.py:145-146
    does, including the axis-aligned and diagonal extremes; the module's own torch restatement agrees
    too; and the Encoding module picks the kernel."""
    from mfnerf import tcnn as T
    from oracle import field_oracle as FO
    g = torch.Generator().manual_seed(5)
    d = torch.randn(100003, 3, generator=g)
    d = torch.cat([d, torch.eye(3), -torch.eye(3), torch.ones(1, 3), -torch.ones(1, 3)])
    d01 = (d / d.norm(dim=-1, keepdim=True) + 1) / 2
    oracle = FO.sh4(d01.float()).half()
    got = T.sh4_fw(d01.to(gpu))
    torch.cuda.synchronize()
    assert got.dtype == torch.float16 and got.shape == (d01.shape[0], 16)
    bad = (got.cpu() != oracle).any(-1).nonzero().flatten()
    assert bad.numel() == 0, (int(bad.numel()), d01[bad[:4]].tolist())
    ref = T.sh4_torch(d01.to(gpu).float()).half()
    assert torch.equal(got, ref)
    enc = T.Encoding(3, {"otype": "SphericalHarmonics", "degree": 4})
    with torch.no_grad():
        assert torch.equal(enc(d01.to(gpu)), ref)

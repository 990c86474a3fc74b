"""The drop-in host path (mfnerf.rendering.render + mfnerf.networks.NGP + mfnerf.losses) on the GPU
against the golden vectors captured from the reference's own Python (tests/golden/make_golden.py).
Marching outputs are bit-exact; field-dependent values carry the fp16 MFMA tolerance."""
import json
import math
import os

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu
GOLD = os.path.join(ROOT, "tests", "golden")


class HP:
    pass


def table_values(n, seed=1):
    """The Lego fixture's table (make_golden.table_values): U(-0.5, 0.5) from a seeded CPU generator."""
    g = torch.Generator().manual_seed(seed)
    return torch.empty(n).uniform_(-0.5, 0.5, generator=g)


@pytest.fixture(scope="module", params=["", "_mf128", "_lego"],
                ids=["hash-rgb64", "mixedfeature-rgb128", "lego-T19-1024rays"])
def setup(gpu, request):
    from mfnerf.networks import NGP
    z = np.load(os.path.join(GOLD, f"golden_render{request.param}.npz"))
    z = {k: torch.from_numpy(z[k]) for k in z.files}
    meta = json.load(open(os.path.join(GOLD, f"golden_render{request.param}.json")))
    hp = HP()
    for k, v in meta["hparams"].items():
        setattr(hp, k, v)
    model = NGP(scale=meta["scale"], hparams=hp).to(gpu)
    with torch.no_grad():
        if request.param == "_lego":  # the real-size table is regenerated, not stored
            n_net = z["xyz_params"].numel()
            model.xyz_encoder.params[:n_net].copy_(z["xyz_params"])
            model.xyz_encoder.params[n_net:].copy_(table_values(model.xyz_encoder.params.numel() - n_net))
        else:
            model.xyz_encoder.params.copy_(z["xyz_params"])
        model.rgb_net.params.copy_(z["rgb_params"])
        model.density_bitfield.copy_(z["bitfield"])
    return z, model


def _blocks(model):
    """(name, lo, hi) of every parameter block: the MLP layers (tcnn layout) and the table levels."""
    from mfnerf.tcnn import mlp_shapes
    out, off = [], 0
    for i, (o, k) in enumerate(mlp_shapes(32, 16, 64, 1)):
        out.append((f"xyz_mlp{i}", off, off + o * k))
        off += o * k
    lay = model.layout
    cuts = sorted(set(lay.offsets))
    for j, o in enumerate(cuts):
        hi = cuts[j + 1] if j + 1 < len(cuts) else lay.n_params // 2
        out.append((f"table@{o}", off + 2 * o, off + 2 * hi))
    rgb, roff = [], 0
    for i, (o, k) in enumerate(mlp_shapes(32, 3, model.rgb_width, 2)):
        rgb.append((f"rgb_mlp{i}", roff, roff + o * k))
        roff += o * k
    return out, rgb


def _check_block(got, ref, name, tol=5e-2):
    """One parameter block's gradient: relative L2 error (fp16 field vs the fp32 reference: ~1% rms)."""
    nr = float(ref.norm())
    if nr == 0:
        assert float(got.abs().max()) == 0, name
        return
    assert float((got - ref).norm()) <= tol * nr, (name, float((got - ref).norm()) / nr)


def test_render_train_vs_golden(gpu, setup):
    from mfnerf import rendering
    from mfnerf.losses import NeRFLoss
    z, model = setup
    N = z["rays_o"].shape[0]
    noise = z["noise"].to(gpu)
    real = torch.rand_like
    torch.rand_like = lambda t, *a, **k: noise.clone() if t.shape == (N,) else real(t, *a, **k)
    try:
        res = rendering.render(model, z["rays_o"].to(gpu), z["rays_d"].to(gpu))
    finally:
        torch.rand_like = real
    n = int(z["rm_samples"])
    assert int(res["rm_samples"]) == n
    assert torch.equal(res["rays_a"].cpu(), z["rays_a"])
    assert torch.equal(res["deltas"].cpu(), z["deltas"]) and torch.equal(res["ts"].cpu(), z["ts"])
    # the field is fp16 (as tcnn): composited values agree to ~1e-3
    assert abs(int(res["vr_samples"]) - int(z["vr_samples"])) <= max(2, n // 500)
    for k in ("opacity", "depth", "rgb"):
        assert torch.allclose(res[k].detach().float().cpu(), z[k], atol=5e-3), k
    loss_d = NeRFLoss(lambda_distortion=0)(res, {"rgb": z["target"].to(gpu)})
    loss = sum(lo.mean() for lo in loss_d.values())
    assert abs(float(loss.detach()) - float(z["loss"])) < 2e-3 * max(1.0, float(z["loss"]))
    model.zero_grad()
    loss.backward()
    # per block (each MLP layer, each table level or shared table): a sign or scale error in one
    # small block cannot hide in the whole vector's cosine
    gx, gr = model.xyz_encoder.params.grad.cpu(), model.rgb_net.params.grad.cpu()
    xyz_blocks, rgb_blocks = _blocks(model)
    for name, lo, hi in rgb_blocks:
        _check_block(gr[lo:hi], z["grad_rgb_params"][lo:hi], name)
    if "grad_xyz_params" in z:
        for name, lo, hi in xyz_blocks:
            _check_block(gx[lo:hi], z["grad_xyz_params"][lo:hi], name)
    else:  # the real-size table: MLP blocks whole, the table on the recorded entries and in norm
        n_net = z["grad_xyz_net"].numel()
        for name, lo, hi in xyz_blocks:
            if hi <= n_net:
                _check_block(gx[lo:hi], z["grad_xyz_net"][lo:hi], name)
        gt = gx[n_net:]
        _check_block(gt[z["grad_table_idx"]], z["grad_table_val"], "table entries")
        assert abs(float(gt.abs().sum()) / float(z["grad_table_l1"]) - 1) < 3e-2
        assert abs(float(gt.norm()) / float(z["grad_table_l2"]) - 1) < 3e-2


def test_render_test_time_vs_golden(gpu, setup):
    from mfnerf import rendering
    z, model = setup
    with torch.no_grad():
        rt = rendering.render(model, z["rays_o"].to(gpu), z["rays_d"].to(gpu), test_time=True)
    assert torch.allclose(rt["opacity"].cpu(), z["test_opacity"], atol=1e-2)
    assert torch.allclose(rt["rgb"].cpu(), z["test_rgb"], atol=1e-2)
    assert abs(int(rt["total_samples"]) - int(z["test_total_samples"])) <= max(4, int(z["test_total_samples"]) // 200)


def test_mark_invisible_cells_vs_golden(gpu, setup):
    z, model = setup
    model.density_grid.zero_()
    model.mark_invisible_cells(z["mark_K"].to(gpu), z["mark_poses"].to(gpu), (100, 100))
    bits = np.packbits((model.density_grid[0] < 0).cpu().numpy(), bitorder="little")
    assert np.array_equal(bits, z["invisible_bits"].numpy())

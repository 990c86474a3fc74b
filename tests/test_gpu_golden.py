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


@pytest.fixture(scope="module", params=["", "_mf128"], ids=["hash-rgb64", "mixedfeature-rgb128"])
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
        model.xyz_encoder.params.copy_(z["xyz_params"])
        model.rgb_net.params.copy_(z["rgb_params"])
        model.density_bitfield.copy_(z["bitfield"])
    return z, model


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
    assert abs(float(loss) - float(z["loss"])) < 2e-3 * max(1.0, float(z["loss"]))
    model.zero_grad()
    loss.backward()
    for got, ref in ((model.xyz_encoder.params.grad, z["grad_xyz_params"]),
                     (model.rgb_net.params.grad, z["grad_rgb_params"])):
        cos = torch.nn.functional.cosine_similarity(got.cpu().flatten(), ref.flatten(), dim=0)
        assert cos > 0.99, float(cos)


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

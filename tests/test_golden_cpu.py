"""The oracle against the golden vectors captured from the reference's own Python host code
(tests/golden/make_golden.py): march, compositing, field, loss and TruncExp on those inputs."""
import json
import math
import os

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import field_oracle as FO

GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module", params=["", "_mf128"], ids=["hash-rgb64", "mixedfeature-rgb128"])
def gold(request):
    z = np.load(os.path.join(GOLD, f"golden_render{request.param}.npz"))
    meta = json.load(open(os.path.join(GOLD, f"golden_render{request.param}.json")))
    return {k: torch.from_numpy(z[k]) for k in z.files}, meta


def _hits(oracle, o, d):
    _, ht, _ = oracle.ray_aabb_intersect(o, d, torch.zeros(1, 3), torch.full((1, 3), 0.5), 1)
    ht[(ht[:, 0, 0] >= 0) & (ht[:, 0, 0] < 0.01), 0, 0] = 0.01  # rendering.py:29
    return ht


def test_oracle_march_matches_golden(gold, oracle):
    z, meta = gold
    ht = _hits(oracle, z["rays_o"], z["rays_d"])
    ra, x, d, de, ts, cnt = oracle.raymarching_train(z["rays_o"], z["rays_d"], ht[:, 0].contiguous(), z["bitfield"],
                                                     1, 0.5, 0.0, z["noise"], 128, 1024)
    n = int(cnt[0])
    assert n == int(z["rm_samples"])
    assert torch.equal(ra, z["rays_a"])
    assert torch.equal(de[:n], z["deltas"]) and torch.equal(ts[:n], z["ts"])


def test_oracle_field_and_composite_match_golden(gold, oracle):
    z, meta = gold
    hp = meta["hparams"]
    b = math.exp(math.log(hp["N_max"] * meta["scale"] / hp["N_min"]) / (hp["L"] - 1))
    lay = FO.GridLayout(hp["L"], hp["F"], hp["T"], hp["N_min"], b, hp["grid"], hp["N_tables"])
    ht = _hits(oracle, z["rays_o"], z["rays_d"])
    ra, x, d, de, ts, cnt = oracle.raymarching_train(z["rays_o"], z["rays_d"], ht[:, 0].contiguous(), z["bitfield"],
                                                     1, 0.5, 0.0, z["noise"], 128, 1024)
    n = int(cnt[0])
    x, d = x[:n], d[:n]
    px = z["xyz_params"]
    feat = FO.grid_encode((x + 0.5) / 1.0, px[3072:], lay)
    h = FO.mlp_forward(feat, px[:3072], 32, 16, 64, 1)
    sigma = torch.exp(h[:, 0])
    dn = d / torch.norm(d, dim=1, keepdim=True)
    rgbs = FO.mlp_forward(torch.cat([FO.sh4((dn + 1) / 2), h], 1), z["rgb_params"], 32, 3, hp["rgb_channels"], 2,
                          "ReLU", "Sigmoid")
    tot, op, dep, rgb, ws = oracle.composite_train_fw(sigma.contiguous(), rgbs.contiguous(), z["deltas"], z["ts"],
                                                      z["rays_a"], 1e-4)
    assert int(tot.sum()) == int(z["vr_samples"])
    assert torch.allclose(op, z["opacity"], atol=1e-5)
    assert torch.allclose(dep, z["depth"], atol=1e-5)
    assert torch.allclose(rgb + (1 - op)[:, None], z["rgb"], atol=1e-5)  # background blend
    e = (rgb + (1 - op)[:, None]) - z["target"]
    o = op + 1e-10
    assert abs(float((e ** 2).mean() + (1e-3 * (-o * torch.log(o))).mean()) - float(z["loss"])) < 1e-6


def test_truncexp_golden(gold):
    z, _ = gold
    x = z["truncexp_x"]
    assert torch.allclose(z["truncexp_y"], torch.exp(x))
    assert torch.allclose(z["truncexp_g"], torch.exp(x.clamp(-15, 15)))

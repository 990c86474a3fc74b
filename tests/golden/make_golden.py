"""Generate the committed golden fixtures by running the REFERENCE's own Python host code.

The reference (lly00412/MF-NeRF, read-only at /root/reference in the build container only) is
imported with its native dependencies replaced by this repo's CPU oracle:
    vren        -> oracle/vren_oracle.py   (C restatement of models/csrc)
    tinycudann  -> oracle/field_oracle.py  (fp32 restatement of the tcnn modules it configures)
    torch_scatter.segment_csr -> a torch restatement (custom_functions.py:107-110)
and driven on seeded synthetic inputs.  What this pins is the reference's HOST semantics around
the kernels: render()'s near clamp and background blend, RayMarcher slicing/outputs,
VolumeRenderer packing (vr_samples), NeRFLoss terms, TruncExp, NGP.forward's normalisation/SH
input/concat order, the test-time progressive loop, mark_invisible_cells, and the gradients the
reference's autograd graph produces.  Only data (inputs/outputs) is written to golden_*.npz.

Run from anywhere:  python tests/golden/make_golden.py [mf128|lego]   (needs /root/reference; CPU only)
"mf128" writes golden_render_mf128.*: the same vectors for the MF benchmark field (MixedFeature
grid with 8 shared tables, rgb_channels 128).
"""
import math
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("MFNERF_REFERENCE", "/root/reference")
sys.dont_write_bytecode = True  # the reference tree is read-only
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]

from oracle import field_oracle, vren_oracle  # noqa: E402


def install_stubs():
    sys.modules["vren"] = vren_oracle
    tc = types.ModuleType("tinycudann")
    tc.Encoding = field_oracle.Encoding
    tc.Network = field_oracle.Network
    tc.NetworkWithInputEncoding = field_oracle.NetworkWithInputEncoding
    sys.modules["tinycudann"] = tc
    ts = types.ModuleType("torch_scatter")

    def segment_csr(src, indptr):
        out = torch.zeros(len(indptr) - 1, *src.shape[1:], dtype=src.dtype)
        seg = torch.repeat_interleave(torch.arange(len(indptr) - 1), indptr[1:] - indptr[:-1])
        return out.index_add_(0, seg, src[indptr[0]:indptr[-1]])

    ts.segment_csr = segment_csr
    sys.modules["torch_scatter"] = ts
    sys.path.insert(0, REF)


class HP:
    """The opt.py fields NGP reads (opt.py:70-90), at a small fixture size."""
    grid, L, F, T, N_min, N_max, N_tables, rgb_channels, rgb_layers = "Hash", 16, 2, 12, 4, 256, 1, 64, 2


class HPMF(HP):
    """The MF benchmark field (benchmark_synthetic_mf.sh: MixedFeature, 8 tables, rgb 128)."""
    grid, N_tables, rgb_channels = "MixedFeature", 8, 128


class HPLego(HP):
    """The Lego training field at its real size (opt.py defaults: Hash L16 F2 T2^19, N_min 16,
    N_max 2048 x scale 0.5 = 1024 finest resolution, rgb 64x2); the 11.4 M-entry table is not
    stored: it is regenerated from TABLE_SEED, and its gradient is recorded per level (L1, L2, max)
    plus on a seeded subset of entries and the largest-magnitude entries."""
    T, N_min, N_max = 19, 16, 2048


TABLE_SEED = 1
N_RAYS = {"": 192, "mf128": 192, "lego": 1024}


def table_values(n, seed=TABLE_SEED):
    """The fixture's table: U(-0.5, 0.5) from a seeded CPU generator (reproducible anywhere)."""
    g = torch.Generator().manual_seed(seed)
    return torch.empty(n).uniform_(-0.5, 0.5, generator=g), g


def main(variant=""):
    global HP
    if variant == "mf128":
        HP = HPMF
    elif variant == "lego":
        HP = HPLego
    install_stubs()
    import warnings
    warnings.filterwarnings("ignore")
    from losses import NeRFLoss
    from models import rendering
    from models.custom_functions import TruncExp
    from models.networks import NGP

    from mfnerf import synthetic

    torch.manual_seed(0)
    scale = 0.5
    model = NGP(scale=scale, hparams=HP)
    G = model.grid_size
    # occupancy: the calibrated ball union (what bench/tests use), packed with the reference's threshold
    grid = synthetic.ball_density_grid(G=G, cascades=model.cascades, scale=scale, seed=3)
    thr = 0.01 * 1024 / math.sqrt(3)
    vren_oracle.packbits(grid.contiguous(), thr, model.density_bitfield)
    # parameters: larger than tcnn's init so the field is not ~constant (fixture is about semantics)
    with torch.no_grad():
        n_net = model.xyz_encoder.n_net
        tab, g = table_values(model.xyz_encoder.params.numel() - n_net)
        model.xyz_encoder.params[n_net:].copy_(tab)
        model.xyz_encoder.params[:n_net].mul_(3)
        model.rgb_net.params.mul_(3)

    poses = synthetic.camera_poses(n_cams=20, seed=2)
    N = N_RAYS[variant]
    rays_o, rays_d = synthetic.random_rays(N, poses, seed=4)
    target = torch.rand(N, 3, generator=g)
    noise = torch.rand(N, generator=g)

    # -- train-mode render (rendering.py:121-163) with the recorded noise (custom_functions.py:83)
    real_rand_like = torch.rand_like
    torch.rand_like = lambda t, *a, **k: noise.clone() if t.shape == (N,) else real_rand_like(t, *a, **k)
    try:
        res = rendering.render(model, rays_o, rays_d)
    finally:
        torch.rand_like = real_rand_like
    loss_d = NeRFLoss(lambda_distortion=0)(res, {"rgb": target})
    loss = sum(lo.mean() for lo in loss_d.values())
    model.zero_grad()
    loss.backward()
    out = {
        "rays_o": rays_o, "rays_d": rays_d, "target": target, "noise": noise,
        "bitfield": model.density_bitfield, "xyz_params": model.xyz_encoder.params.detach(),
        "rgb_params": model.rgb_net.params.detach(),
        "rays_a": res["rays_a"], "deltas": res["deltas"], "ts": res["ts"],
        "rm_samples": torch.tensor(int(res["rm_samples"])), "vr_samples": res["vr_samples"].detach(),
        "opacity": res["opacity"].detach(), "depth": res["depth"].detach(), "rgb": res["rgb"].detach(),
        "ws": res["ws"].detach(), "loss": loss.detach(), "loss_rgb": loss_d["rgb"].mean().detach(),
        "loss_opacity": loss_d["opacity"].mean().detach(),
        "grad_xyz_params": model.xyz_encoder.params.grad, "grad_rgb_params": model.rgb_net.params.grad,
    }
    # -- test-mode render (rendering.py:46-118), progressive loop
    with torch.no_grad():
        rt = rendering.render(model, rays_o, rays_d, test_time=True)
    out.update({"test_opacity": rt["opacity"], "test_depth": rt["depth"], "test_rgb": rt["rgb"],
                "test_total_samples": torch.tensor(int(rt["total_samples"]))})
    # -- TruncExp fw/bw (custom_functions.py:162-173) incl. the clamp
    x = torch.tensor([-30.0, -15.0, -1.0, 0.0, 2.0, 15.0, 30.0], requires_grad=True)
    y = TruncExp.apply(x)
    y.sum().backward()
    out.update({"truncexp_x": x.detach(), "truncexp_y": y.detach(), "truncexp_g": x.grad})
    # -- mark_invisible_cells (networks.py:199-240): cameras that see part of the box
    K = torch.tensor([[synthetic.LEGO_F / 8, 0, 50.0], [0, synthetic.LEGO_F / 8, 50.0], [0, 0, 1]])
    model.density_grid = torch.zeros(model.cascades, G ** 3)
    model.register_buffer("grid_coords", torch.stack(torch.meshgrid(*[torch.arange(G, dtype=torch.int32)] * 3,
                                                                    indexing="ij"), -1).reshape(-1, 3))
    model.mark_invisible_cells(K, poses[:3], (100, 100))
    out["invisible_bits"] = torch.from_numpy(np.packbits((model.density_grid[0] < 0).numpy(), bitorder="little"))
    out["mark_K"], out["mark_poses"] = K, poses[:3]

    if variant == "lego":  # the table and its gradient are too large to store whole
        gt = out.pop("grad_xyz_params")
        out["xyz_params"] = out["xyz_params"][:n_net].clone()
        out["grad_xyz_net"] = gt[:n_net].clone()
        gtab = gt[n_net:]
        sub = torch.randperm(gtab.numel(), generator=torch.Generator().manual_seed(5))[:65536]
        top = gtab.abs().topk(4096).indices
        idx = torch.cat([sub, top]).unique()
        out["grad_table_idx"], out["grad_table_val"] = idx, gtab[idx].clone()
        out["grad_table_l1"], out["grad_table_l2"] = gtab.abs().sum(), gtab.norm()
    tag = "_" + variant if variant else ""
    np.savez_compressed(os.path.join(HERE, f"golden_render{tag}.npz"),
                        **{k: v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v) for k, v in out.items()})
    meta = {"hparams": {k: getattr(HP, k) for k in ("grid", "L", "F", "T", "N_min", "N_max", "N_tables",
                                                    "rgb_channels", "rgb_layers")}, "scale": scale, "n_rays": N}
    import json
    with open(os.path.join(HERE, f"golden_render{tag}.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"wrote golden_render{tag}.npz:", {k: tuple(v.shape) for k, v in out.items() if isinstance(v, torch.Tensor)})


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "")

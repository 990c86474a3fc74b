"""Seed-to-seed spread of the training-parity protocol on this repo's GPU step (tests/parity_protocol.py):
trains K runs (batch/perturbation seeds 0..K-1, same initial weights) and prints each held-out PSNR.
    python tools/parity_spread.py [K]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import parity_protocol as PP  # noqa: E402
from mfnerf import engine  # noqa: E402
from mfnerf.rendering import render  # noqa: E402
from test_gpu_parity_train import _ngp  # noqa: E402


def run(seed, dev):
    cfg = PP.config()
    st = engine.TrainStep(cfg, device=dev, seed=PP.INIT_SEED)
    st.set_occupancy(PP.density_grid())
    train, test = PP.scene()
    for step in range(PP.STEPS):
        if step % PP.STEPS_PER_EPOCH == 0:
            st.set_lr(PP.lr_at(step))
        o, d, rgb = PP.batch(train, step, seed)
        st.run(engine.Batch(o.to(dev), d.to(dev), rgb.to(dev)), noise=PP.noise(step, seed).to(dev))
    model = _ngp(st, cfg)
    imgs, poses, dirs, _ = test
    views = []
    with torch.no_grad():
        for img, pose in zip(imgs, poses):
            o = pose[:, 3].expand(dirs.shape[0], 3).contiguous().to(dev)
            dd = (dirs @ pose[:, :3].T).contiguous().to(dev)
            views.append(PP.psnr(render(model, o, dd, test_time=True)["rgb"].cpu(), img))
    return sum(views) / len(views)


if __name__ == "__main__":
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device("cuda:0")
    ps = [run(s, dev) for s in range(k)]
    m = sum(ps) / k
    sd = (sum((p - m) ** 2 for p in ps) / max(1, k - 1)) ** 0.5
    print(f"epochs {PP.EPOCHS} x {PP.STEPS_PER_EPOCH} steps, {PP.N_TEST} views: PSNR per seed",
          [round(p, 3) for p in ps], "mean", round(m, 3), "std", round(sd, 3), flush=True)

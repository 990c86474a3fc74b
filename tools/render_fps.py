"""Test-time rendering speed of the drop-in path (the reference's README.md:123
quotes 36.20 FPS for Lego 800x800 on an RTX 2080 Ti).

Trains the field on the analytic ball scene (mfnerf.data, Lego intrinsics) for --train-steps
steps with the fused trainer, then times mfnerf.rendering.render(test_time=True) -- the reference's
progressive test-time loop (rendering.py:46-118) over raymarching_test / composite_test_fw -- on
full 800x800 held-out views, and reports frames/s and PSNR.  One JSON line on stdout.

    python tools/render_fps.py [--train-steps 2000] [--views 5]
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--train-steps", type=int, default=2000)
    ap.add_argument("--views", type=int, default=5)
    ap.add_argument("--width", type=int, default=800)
    args = ap.parse_args()
    from mfnerf import data, synthetic
    from mfnerf.rendering import render
    from mfnerf.trainer import HParams, Trainer

    dev = torch.device("cuda:0")
    W = args.width
    focal = 0.5 * W / math.tan(0.5 * 0.6911112)  # Lego field of view
    scene = data.BallScene.matching_grid(seed=0)
    imgs, poses, dirs, K = data.ball_scene_views(scene, 50, W, focal, seed=0, device=dev)
    ds = data.DeviceDataset(imgs, poses, dirs, K=K, img_wh=(W, W), device=dev, seed=1)
    del imgs
    hp = HParams(batch_size=8192, num_epochs=1, steps_per_epoch=args.train_steps)
    tr = Trainer(hp, ds, device=dev)
    t0 = time.time()
    tr.fit(log_every=0)
    torch.cuda.synchronize()
    train_s = time.time() - t0
    model = tr.to_ngp()
    t_imgs, t_poses, _, _ = data.ball_scene_views(scene, args.views, W, focal, seed=11, device=dev)
    dd = dirs.to(dev)
    times, psnrs, samples = [], [], []
    with torch.no_grad():
        for i, (img, pose) in enumerate(zip(t_imgs, t_poses)):
            o, d = data.get_rays(dd, pose.to(dev))
            torch.cuda.synchronize()
            t = time.time()
            res = render(model, o, d, test_time=True)
            torch.cuda.synchronize()
            if i > 0 or args.views == 1:  # the first frame warms up allocations
                times.append(time.time() - t)
            psnrs.append(float(-10 * torch.log10(((res["rgb"].float() - img) ** 2).mean())))
            samples.append(int(res["total_samples"]))
    fps = len(times) / sum(times)
    print(json.dumps({"metric": "test-time render frames/s (800x800)", "fps": round(fps, 2),
                      "ms_per_frame": round(1e3 / fps, 2), "psnr": round(sum(psnrs) / len(psnrs), 2),
                      "samples_per_ray": round(sum(samples) / len(samples) / (W * W), 2),
                      "train_steps": args.train_steps, "train_s": round(train_s, 2), "views": args.views,
                      "reference": "36.20 FPS, RTX 2080 Ti, Lego (README.md:123)",
                      "data": "analytic 12-ball scene, Lego intrinsics (no dataset in the image)"}), flush=True)


if __name__ == "__main__":
    main()

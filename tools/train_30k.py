"""The reference's Lego training protocol end to end on one GPU: train.py defaults (30 epochs x 1000
steps, 8192 rays/batch, Hash L16 F2 T2^19, lr 1e-2 cosine, occupancy refresh every 16 steps with
the 256-step warm-up, train.py:53-245) over 100 analytic 800x800 views, then the test PSNR of held-out
views with the test-time renderer (train.py:197-206).  The Lego images are not in the image, so the
scene is the bench's 12-ball scene with a world-space surface texture (detail for the fine levels).

Prints one JSON line: training wall time (occupancy refreshes, lr steps and logging included),
whole-run rays/s, per-1000-step train PSNR / rm_s, and the test PSNR.

    python tools/train_30k.py [--epochs 30] [--tex 40] [--views 100] [--test-views 8]
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]
# graph replays through the per-node launch path, as bench.py (before the HIP runtime initialises)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
import torch  # noqa: E402

from mfnerf import data, synthetic  # noqa: E402
from mfnerf.trainer import HParams, Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=30)
    ap.add_argument("--steps-per-epoch", type=int, default=1000)
    ap.add_argument("--tex", type=float, default=40.0, help="surface texture frequency (0 = flat colours)")
    ap.add_argument("--views", type=int, default=100)
    ap.add_argument("--test-views", type=int, default=8)
    ap.add_argument("--W", type=int, default=synthetic.LEGO_W)
    ap.add_argument("--grid", default="Hash")
    ap.add_argument("--T", type=int, default=19)
    ap.add_argument("--mf", action="store_true",
                    help="benchmark_synthetic_nerf_mf.sh's field and schedule: MixedFeature 8 tables, T2^20, "
                         "rgb 128, 16384 rays, lr 2e-2, 20 epochs")
    args = ap.parse_args()
    dev = torch.device("cuda")
    W = args.W
    focal = 0.5 * W / math.tan(0.5 * 0.6911112)
    scene = data.BallScene.matching_grid(seed=0)
    scene.texture_freq = args.tex
    imgs, poses, dirs, K = data.ball_scene_views(scene, args.views, W, focal, seed=0, device=dev)
    t_imgs, t_poses, _, _ = data.ball_scene_views(scene, args.test_views, W, focal, seed=7, device=dev)
    ds = data.DeviceDataset(imgs, poses, dirs, K=K, img_wh=(W, W), device=dev, seed=5)
    if args.mf:
        hp = HParams(num_epochs=20, steps_per_epoch=args.steps_per_epoch, grid="MixedFeature", N_tables=8, T=20,
                     rgb_channels=128, batch_size=16384, lr=2e-2)
    else:
        hp = HParams(num_epochs=args.epochs, steps_per_epoch=args.steps_per_epoch, grid=args.grid, T=args.T)
    tr = Trainer(hp, ds, device=dev)
    hist = []

    def log(m):
        hist.append(m)
        print(f"step {m['step']:6d}  loss {m['loss']:.5f}  train psnr {m['psnr']:.2f}  rm_s {m['rm_s']:.1f}  "
              f"lr {m['lr']:.2e}  overflowed records {m['overflow_records']}  t {time.perf_counter() - t0:.1f}s",
              flush=True)

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.fit(log_every=args.steps_per_epoch, log=log)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    steps = tr.global_step
    t1 = time.perf_counter()
    test_psnr, per_view = tr.evaluate(t_imgs, t_poses, dirs)
    eval_s = time.perf_counter() - t1
    white = sum(float(-10 * torch.log10(((1 - im) ** 2).mean())) for im in t_imgs) / len(t_imgs)
    print(json.dumps({
        "protocol": f"{'benchmark_synthetic_nerf_mf.sh' if args.mf else 'train.py defaults'}: {steps} steps x "
                    f"{hp.batch_size} rays, {hp.grid} L{hp.L} F{hp.F} T2^{hp.T}"
                    f"{' %d tables' % hp.N_tables if hp.grid == 'MixedFeature' else ''}, rgb {hp.rgb_channels}, "
                    f"lr {hp.lr} cosine, occupancy every 16 steps",
        "scene": f"12-ball scene (bench occupancy balls), texture_freq {args.tex}, {args.views} train / "
                 f"{args.test_views} held-out views at {W}x{W}, Lego intrinsics",
        "train_wall_s": round(wall, 2), "rays_per_s_whole_run": round(steps * hp.batch_size / wall, 1),
        "test_psnr": round(test_psnr, 3), "test_psnr_per_view": [round(v, 3) for v in per_view],
        "white_image_psnr": round(white, 3), "eval_s": round(eval_s, 2), "skipped_steps": hist[-1]["skipped"],
        # records the partitioned scatter's slots could not hold (added by atomics), per logged
        # interval of steps_per_epoch steps and in total
        "overflow_records_total": hist[-1]["overflow_records"],
        "overflow_records_per_interval": [b["overflow_records"] - a["overflow_records"]
                                          for a, b in zip([{"overflow_records": 0}] + hist[:-1], hist)],
        "train_log": [{k: (round(v, 4) if isinstance(v, float) else v) for k, v in h.items()} for h in hist],
        "device": torch.cuda.get_device_name(0)}))


if __name__ == "__main__":
    main()

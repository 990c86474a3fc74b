"""Diagnose train-vs-test PSNR of the trainer on the ball scene (GPU)."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]
import torch  # noqa: E402

from mfnerf import data  # noqa: E402
from mfnerf.rendering import render  # noqa: E402
from mfnerf.trainer import HParams, Trainer, psnr  # noqa: E402

W = 64
focal = 0.5 * W / math.tan(0.5 * 0.6911112)
scene = data.BallScene(n_balls=6, seed=1)
imgs, poses, dirs, K = data.ball_scene_views(scene, 100, W, focal, seed=0)
t_imgs, t_poses, _, _ = data.ball_scene_views(scene, 4, W, focal, seed=7)
dev = torch.device("cuda")
ds = data.DeviceDataset(imgs, poses, dirs, K=K, img_wh=(W, W), device=dev, seed=5)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 600
hp = HParams(batch_size=4096, T=int(os.environ.get("T", 16)), num_epochs=1, steps_per_epoch=steps)
tr = Trainer(hp, ds, device=dev, graphs=os.environ.get("GRAPHS", "1") == "1")
hist = tr.fit(log_every=200)
print("train hist", [(h["step"], round(h["psnr"], 1), round(h["rm_s"], 1)) for h in hist])
m = tr.to_ngp()
for name, I, P in (("train views", imgs[:4], poses[:4]), ("test views", t_imgs, t_poses)):
    for mode in (True, False):
        vals = []
        for img, pose in zip(I, P):
            o, d = data.get_rays(dirs.to(dev), pose.to(dev))
            with torch.no_grad():
                r = render(m, o, d, test_time=mode)
            vals.append(psnr(r["rgb"].float(), img.to(dev)))
        print(f"{name:12s} {'test-time' if mode else 'train-mode'} renderer: {[round(v, 2) for v in vals]}")
# engine's own prediction on a full training image through the training path (eager run on a fixed batch)
st = tr.step
o, d = data.get_rays(dirs.to(dev), poses[0].to(dev))
from mfnerf.engine import Batch
b = Batch(o.contiguous(), d.contiguous(), imgs[0].to(dev).contiguous())
st.cfg.lr = 0.0
st.set_lr(0.0)
if st.cfg.n_rays == o.shape[0]:
    st.run(b)
    pred = torch.cat([t.rgb + (1 - t.opacity)[:, None] for t in st.parts])
    print("engine train-path PSNR on train view 0:", round(psnr(pred, b.rgb), 2))

# a sampled batch vs the same rays rebuilt on the host from the sampled indices
N = st.cfg.n_rays
buf = torch.empty(3, N, 3, device=dev)
ii = torch.empty(N, dtype=torch.int32, device=dev)
pp = torch.empty(N, dtype=torch.int32, device=dev)
ds.sample(buf, ii, pp)
ic, pc = ii.long().cpu(), pp.long().cpu()
o2, d2 = data.get_rays(dirs[pc], poses[ic])
print("sampled vs host rays: max|do|", float((buf[0].cpu() - o2).abs().max()), "max|dd|",
      float((buf[1].cpu() - d2).abs().max()), "rgb equal", bool(torch.equal(buf[2].cpu(), imgs[ic, pc])))
print("non-white fraction: sampled gt", float((buf[2] < 0.999).any(-1).float().mean()),
      "images", float((imgs < 0.999).any(-1).float().mean()))
from mfnerf.engine import _packed_batch
sb = _packed_batch(buf)
st.run(sb)
pred = torch.cat([t.rgb + (1 - t.opacity)[:, None] for t in st.parts])
print("engine PSNR on a sampled batch:", round(psnr(pred, sb.rgb), 2))
hb = Batch(o2.to(dev).contiguous(), d2.to(dev).contiguous(), imgs[ic, pc].to(dev).contiguous())
st.run(hb)
pred = torch.cat([t.rgb + (1 - t.opacity)[:, None] for t in st.parts])
print("engine PSNR on the host-built same rays:", round(psnr(pred, hb.rgb), 2))

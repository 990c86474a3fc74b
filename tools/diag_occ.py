"""Diagnostics of the engine's occupancy refresh vs the restated update (GPU)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]
import torch  # noqa: E402

from mfnerf import engine, synthetic  # noqa: E402
from oracle import occupancy_oracle as OO  # noqa: E402

gpu = torch.device("cuda:0")
st = engine.TrainStep(engine.StepConfig(n_rays=512, log2_T=16), device=gpu, seed=0)
st.set_occupancy(synthetic.ball_density_grid())
poison = "--poison" in sys.argv  # fill the refresh's buffers with garbage first (uninitialised reads)
st.update_density_grid(warmup=True)  # allocates the buffers
st.set_occupancy(synthetic.ball_density_grid())
for warm in (True, False, False):
    before = st.density_grid.clone().cpu()
    if poison:
        o = st._occ
        o.sigma.fill_(1.5e27)
        o.xyz.fill_(float("nan"))
        o.cell.fill_(12345)
        o.feat.fill_(float("nan"))
    st.update_density_grid(warmup=warm)
    torch.cuda.synchronize()
    o = st._occ
    n = int(o.count)
    cell = o.cell[:n].cpu().long()
    sig = o.sigma[:n].cpu()
    ref_g, thr, _ = OO.update(before, sig, cell.int())
    got = st.density_grid.cpu()
    bad = (got != ref_g).reshape(-1).nonzero().flatten()
    tmp = o.tmp.cpu()
    pos = torch.full((got.numel(),), -1, dtype=torch.long)
    pos[cell] = torch.arange(n)
    print(f"warm={warm} n={n} sigma finite={bool(torch.isfinite(sig).all())} max={float(sig.max()):.4g} "
          f"mismatches={bad.numel()} sorted={bool((cell[1:] > cell[:-1]).all())}", flush=True)
    for k in bad[:8].tolist():
        i = int(pos[k])
        print(f"  cell {k}: got {float(got.reshape(-1)[k]):.6g} ref {float(ref_g.reshape(-1)[k]):.6g} before "
              f"{float(before.reshape(-1)[k]):.6g} tmp {float(tmp[k]):.6g} list index {i} "
              f"sigma {float(sig[i]) if i >= 0 else float('nan'):.6g}", flush=True)

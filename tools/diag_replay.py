import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "mf-nerf_amd")]
import torch
from mfnerf import engine, synthetic
gpu = torch.device("cuda:0")
def mk():
    st = engine.TrainStep(engine.StepConfig(n_rays=1024, log2_T=16, n_parts=1), device=gpu, seed=0)
    st.set_occupancy(synthetic.ball_density_grid()); return st
K = 4
a, b = mk(), mk()
batches = a.make_batches(K + 1, seed=3)
ref = []
for k in range(K):
    b.run(batches[k]); torch.cuda.synchronize(); ref.append((b.params.clone(), b.m.clone()))
a.run(batches[0]); torch.cuda.synchronize(); got = [(a.params.clone(), a.m.clone())]
a.capture()
for k in range(1, K):
    a.replay(batches[k], next_batch=batches[k + 1] if k + 1 < K else None); torch.cuda.synchronize()
    got.append((a.params.clone(), a.m.clone()))
for k in range(K):
    for name, x, y in (("params", got[k][0], ref[k][0]), ("m", got[k][1], ref[k][1])):
        d = (x != y).nonzero()[:, 0]
        blocks = [(0, a.off_rgb), (a.off_rgb, a.off_table), (a.off_table, a.n_alloc)]
        print(k, name, "ndiff", d.numel(), "per block", [int(((d >= lo) & (d < hi)).sum()) for lo, hi in blocks],
              "maxabs", float((x - y).abs().max()))

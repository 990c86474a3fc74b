"""Attribute grid_bw time: product vs plain-store body vs level subsets, on the bench workload."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]
import torch
import bench
from mfnerf import engine, synthetic
from mfnerf._lib import call, ptr, stream
dev = torch.device("cuda:0")
step = engine.TrainStep(engine.StepConfig(), device=dev)
step.set_occupancy(synthetic.ball_density_grid())
b = step.make_batches(2, seed=100)
for i in range(5):
    bench.run_step(step, b[i % 2], 1)
torch.cuda.synchronize()
mb, part = step.state.march.part[0], step.parts[0]
for mode in (0, 1, 2, 3, 0):
    ts = []
    for rep in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        call("mfnerf_debug_grid_bw_ablate", mode, ptr(mb.xyzs), step.cap_p, ptr(mb.counter), step.x_min,
             step.x_range, step.desc, ptr(part.dfeat), ptr(step.grads[step.off_table:]), stream())
        e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    ts.sort()
    print(f"mode {mode}: median {ts[10]*1e3:.1f} us  min {ts[0]*1e3:.1f} us", flush=True)
# the product call (with the dense-level private copies + fold)
ts = []
for rep in range(20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    step._grid_bw(step.state.march, 0)
    e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
ts.sort()
print(f"product (copies+fold): median {ts[10]*1e3:.1f} us  min {ts[0]*1e3:.1f} us", flush=True)

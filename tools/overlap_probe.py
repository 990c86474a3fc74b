"""Do back-to-back launches of grid_bw (eager or graph) overlap?  Timing + a lost-update check."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]
import torch  # noqa: E402

from mfnerf import engine, synthetic  # noqa: E402

st = engine.TrainStep(engine.StepConfig(), device="cuda")
st.set_occupancy(synthetic.ball_density_grid())
bs = st.make_batches(8)
for i in range(5):
    st.run(bs[i % 8])
st.capture()
torch.cuda.synchronize()
tab = st.grads[st.off_table:]


def wall(fn, k=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


print("eager grid_bw back-to-back  ms", wall(st._grid_bw))
print("graph grid_bw back-to-back  ms", wall(lambda: st.graphs["grid_bw"].replay()))
e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
e[0].record()
for _ in range(20):
    st.graphs["grid_bw"].replay()
e[1].record()
torch.cuda.synchronize()
print("graph grid_bw events/20     ms", e[0].elapsed_time(e[1]) / 20)

# lost updates: 1 launch vs 10 launches accumulate 10x the same gradient
tab.zero_()
st._grid_bw()
torch.cuda.synchronize()
one = tab.double().sum().item(), tab.abs().double().sum().item()
for name, fn in (("eager", st._grid_bw), ("graph", lambda: st.graphs["grid_bw"].replay())):
    tab.zero_()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    ten = tab.double().sum().item(), tab.abs().double().sum().item()
    print(name, "10x/1x sum ratio", ten[0] / one[0], "abs ratio", ten[1] / one[1])

"""grid_bw duration vs the cache state of the gradient table (GPU diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]
import torch  # noqa: E402

from mfnerf import engine, synthetic  # noqa: E402

st = engine.TrainStep(engine.StepConfig(), device="cuda")
st.set_occupancy(synthetic.ball_density_grid())
bs = st.make_batches(8)
for i in range(10):
    st.run(bs[i % 8])
torch.cuda.synchronize()
flush = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
tab = st.grads[st.off_table:]


def t_grid_bw(pre, k=20):
    ts = []
    for _ in range(k):
        pre()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        st._grid_bw()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


print("hot (repeat)            ", t_grid_bw(lambda: None))
print("after 1 GB flush        ", t_grid_bw(lambda: flush.fill_(1)))
print("flush + zero table      ", t_grid_bw(lambda: (flush.fill_(1), tab.zero_())))
print("flush + read table      ", t_grid_bw(lambda: (flush.fill_(1), tab.sum())))
print("flush + zero all grads  ", t_grid_bw(lambda: (flush.fill_(1), st.grads.zero_())))
print("flush + read dfeat/xyz  ", t_grid_bw(lambda: (flush.fill_(1), st.state.dfeat.sum(), st.state.xyzs.sum())))
print("flush+zero tab+read dfeat", t_grid_bw(lambda: (flush.fill_(1), tab.zero_(), st.state.dfeat.sum())))
print("adam then grid_bw       ", t_grid_bw(lambda: st._update()))
print("adam, zero tab, grid_bw ", t_grid_bw(lambda: (st._update(), tab.zero_())))
n = int(st.state.counter[0])
print("samples", n)

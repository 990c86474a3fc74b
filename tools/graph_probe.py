"""Where does the inter-graph gap come from?  Host time per launch call vs device step time for
eager, 3-segment graphs, and a single whole-step graph (GPU only, diagnostic)."""
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
for i in range(10):
    st.run(bs[i % 8])
st.capture()
g1 = torch.cuda.CUDAGraph()
g1.register_generator_state(st.gen)
with torch.cuda.graph(g1, pool=torch.cuda.graph_pool_handle()):
    st._fwbw(st._static, lambda n: None)
    st._grid_bw()
    st._update()
torch.cuda.synchronize()


def timeit(name, fn, k=200):
    for i in range(10):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        fn(i)
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    print(f"{name:28s} host {th / k * 1e3:7.3f} ms/step   wall {t / k * 1e3:7.3f} ms/step", flush=True)


timeit("eager", lambda i: st.run(bs[i % 8]))
timeit("3 graphs", lambda i: st.replay(bs[i % 8]))
timeit("3 graphs, no copy", lambda i: [st.graphs[n].replay() for n in ("fwbw", "grid_bw", "update")])


def one(i):
    st._static.buf.copy_(bs[i % 8].buf)
    g1.replay()


timeit("1 graph", one)
timeit("1 graph, no copy", lambda i: g1.replay())
timeit("grid_bw graph only", lambda i: st.graphs["grid_bw"].replay())
timeit("fwbw graph only", lambda i: st.graphs["fwbw"].replay())

"""Can timing events be recorded inside a captured HIP graph (ROCm)?  And how large is the gap of
3 graph launches vs 1 (same batches, alternating, same process)?"""
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
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
g1 = torch.cuda.CUDAGraph()
g1.register_generator_state(st.gen)
ok = True
try:
    with torch.cuda.graph(g1, pool=torch.cuda.graph_pool_handle()):
        st._fwbw(st._static, lambda n: None)
        ev[0].record()
        st._grid_bw()
        ev[1].record()
        st._update()
    torch.cuda.synchronize()
except Exception as e:  # noqa: BLE001
    ok = False
    print("capture with events failed:", repr(e))
if ok:
    for i in range(3):
        st._static.buf.copy_(bs[i].buf)
        g1.replay()
        torch.cuda.synchronize()
        try:
            print("in-graph grid_bw event ms:", ev[0].elapsed_time(ev[1]))
        except Exception as e:  # noqa: BLE001
            print("elapsed_time failed:", repr(e))


def loop(fn, k=100):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        fn(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


def one(i):
    st._static.buf.copy_(bs[i % 8].buf)
    g1.replay()


for rep in range(3):
    print("3 graphs ms/step", loop(lambda i: st.replay(bs[i % 8])), " 1 graph ms/step", loop(one))

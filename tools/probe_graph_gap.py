"""Probe: the GPU-side gap between consecutive HIP graph replays (the training step's ~21 us
graph-to-graph gap).  Times R replays of a graph holding K copies of one ~10 us kernel, against
R*K eager launches, and prints the per-replay overhead.  Run it under different runtime
environment settings to see which, if any, shortens the gap.

    python tools/probe_graph_gap.py"""
import json
import os

import torch


def main():
    dev = torch.device("cuda:0")
    x = torch.ones(8 << 20, device=dev)  # 32 MB: one elementwise pass ~10 us
    def work():
        x.mul_(1.0000001)
    for _ in range(10):
        work()
    torch.cuda.synchronize()
    out = {"env": {k: v for k, v in os.environ.items() if k.startswith(("HIP_", "DEBUG_CLR", "AMD_", "GPU_"))}}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    R = 200
    e0.record()
    for _ in range(R * 4):
        work()
    e1.record()
    torch.cuda.synchronize()
    out["eager_us_per_kernel"] = e0.elapsed_time(e1) * 1e3 / (R * 4)
    for K in (1, 2, 4):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            work()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            for _ in range(K):
                work()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(R):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1e3 / R
        out[f"graph_K{K}_us_per_replay"] = t
        out[f"graph_K{K}_gap_us"] = t - K * out["eager_us_per_kernel"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()

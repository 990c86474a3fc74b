"""Probe: do torch external events recorded inside a captured HIP graph time the graph's work?"""
import torch

dev = torch.device("cuda:0")
x = torch.randn(4096, 4096, device=dev)
y = torch.empty_like(x)
e0 = torch.cuda.Event(enable_timing=True, external=True)
e1 = torch.cuda.Event(enable_timing=True, external=True)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    y.copy_(x @ x)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
with torch.cuda.graph(g):
    y.copy_(x @ x)
    e0.record()
    for _ in range(5):
        y.copy_(x @ x)
    e1.record()
    y.copy_(x @ x)
for i in range(3):
    g.replay()
    torch.cuda.synchronize()
    print("replay", i, "inner ms", e0.elapsed_time(e1))
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(5):
    y.copy_(x @ x)
b.record()
torch.cuda.synchronize()
print("eager 5 matmuls ms", a.elapsed_time(b))

"""Probe: hipEventRecordWithFlags(hipEventRecordExternal) inside a torch-captured HIP graph -- does
each replay re-record the events so that hipEventElapsedTime times the graph's inner work?"""
import ctypes

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
hip.hipEventRecordWithFlags.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]


def ev():
    e = ctypes.c_void_p()
    assert hip.hipEventCreate(ctypes.byref(e)) == 0
    return e


dev = torch.device("cuda:0")
x = torch.randn(4096, 4096, device=dev)
y = torch.empty_like(x)
e0, e1 = ev(), ev()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    y.copy_(x @ x)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    y.copy_(x @ x)
    st = torch.cuda.current_stream().cuda_stream
    print("record rc", hip.hipEventRecordWithFlags(e0, st, 1))
    for _ in range(5):
        y.copy_(x @ x)
    print("record rc", hip.hipEventRecordWithFlags(e1, st, 1))
    y.copy_(x @ x)
for n in (1, 3):
    for i in range(n):
        g.replay()
    torch.cuda.synchronize()
    ms = ctypes.c_float()
    rc = hip.hipEventElapsedTime(ctypes.byref(ms), e0, e1)
    print("after", n, "replays: rc", rc, "inner ms", ms.value)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(5):
    y.copy_(x @ x)
b.record()
torch.cuda.synchronize()
print("eager 5 matmuls ms", a.elapsed_time(b))

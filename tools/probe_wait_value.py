"""Probe (GPU box): does hipStreamWaitValue32 on plain device memory hold a stream until a kernel on
another stream writes the value -- without a resident polling wave?  The gated march could then
start at the step graph's gate signal with no gate_wait_kernel spinning beside the chain.

    python tools/probe_wait_value.py
Prints the wait's release time against the writer's, for a few delays.
"""
import ctypes
import os

import torch

HIP_WAIT_GTE = 0x0


def main():
    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    f = lib.hipStreamWaitValue32
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint, ctypes.c_uint32]
    f.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    flag = torch.zeros(4, dtype=torch.int32, device=dev)
    x = torch.zeros(1024, device=dev)
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    for target, cycles in ((1, 2_000_000), (2, 20_000_000), (3, 200_000)):
        e0, ea, eb = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        with torch.cuda.stream(a):
            e0.record(a)
            torch.cuda._sleep(cycles)
            flag[0].fill_(target)
            ea.record(a)
        rc = f(ctypes.c_void_p(b.cuda_stream), ctypes.c_void_p(flag.data_ptr()), target, HIP_WAIT_GTE, 0xFFFFFFFF)
        with torch.cuda.stream(b):
            x.add_(1.0)
            eb.record(b)
        torch.cuda.synchronize()
        print(f"target {target} sleep {cycles}: rc {rc}; writer done at {e0.elapsed_time(ea):.3f} ms, "
              f"waiter's kernel done at {e0.elapsed_time(eb):.3f} ms (must be >= the writer's)", flush=True)
    # the same inside a captured graph: can the wait be a node?
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    try:
        with torch.cuda.stream(s):
            g.capture_begin()
            rc = f(ctypes.c_void_p(s.cuda_stream), ctypes.c_void_p(flag.data_ptr()), 4, HIP_WAIT_GTE, 0xFFFFFFFF)
            x.add_(1.0)
            g.capture_end()
        print("capture: rc", rc, flush=True)
        flag[0].fill_(4)
        g.replay()
        torch.cuda.synchronize()
        print("captured wait replayed", flush=True)
    except Exception as e:  # noqa: BLE001
        print("capture failed:", type(e).__name__, e, flush=True)


if __name__ == "__main__":
    main()

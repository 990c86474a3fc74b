"""A direct RCCL communicator for the data-parallel step: the gradient reduce-scatter,
the fp16 all-gather and the all-reduce issued with ncclReduceScatter / ncclAllGather / ncclAllReduce
on the CALLER's HIP stream.  Issued that way they are plain nodes of the step's HIP graph when
captured (torch.distributed runs RCCL on an internal stream joined by events, which a capture turns
into cross-stream edges), so the whole data-parallel step replays as ONE graph: no host hop between
the backward, the exchange and the sharded Adam (the reference's DDP path, train.py:277-287, overlaps
bucketed all-reduces with the backward on NCCL's stream; here the step is one device-side sequence).

The library is the librccl.so torch already loaded (one RCCL instance per process); the unique id
travels over the existing torch.distributed process group (any backend).
"""
import ctypes
import os

import torch
import torch.distributed as dist

NCCL_FLOAT16, NCCL_FLOAT32 = 6, 7
NCCL_SUM, NCCL_AVG = 0, 4


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        lib = ctypes.CDLL(path if os.path.exists(path) else "librccl.so")
        lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId, ctypes.c_int]
        lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        lib.ncclGetErrorString.restype = ctypes.c_char_p
        lib.ncclGetErrorString.argtypes = [ctypes.c_int]
        for f in ("ncclReduceScatter", "ncclAllReduce"):
            getattr(lib, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p]
        lib.ncclAllGather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p]
        _LIB = lib
    return _LIB


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: RCCL error {rc} ({_lib().ncclGetErrorString(rc).decode()})")


def _dtype(t):
    if t.dtype == torch.float32:
        return NCCL_FLOAT32
    if t.dtype == torch.float16:
        return NCCL_FLOAT16
    raise TypeError(f"RCCL exchange of {t.dtype} is not used by the step")


class Comm:
    """One RCCL communicator over the ranks of the default torch.distributed group (this rank's
    current HIP device).  Collectives are stream-ordered on torch's current stream."""

    def __init__(self):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("rccl.Comm needs an initialised torch.distributed process group")
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        lib = _lib()
        uid = _UniqueId()
        if self.rank == 0:
            _check(lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        # the raw 128 bytes (the c_char array field would stop at the first NUL byte)
        box = [ctypes.string_at(ctypes.addressof(uid), 128) if self.rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        if len(box[0]) != 128:
            raise RuntimeError("rccl.Comm: malformed unique id")
        uid = _UniqueId.from_buffer_copy(box[0])
        self.comm = ctypes.c_void_p()
        torch.cuda.synchronize()
        _check(lib.ncclCommInitRank(ctypes.byref(self.comm), self.world, uid, self.rank), "ncclCommInitRank")
        # the mean's reduction op: at one rank the mean IS the sum, and RCCL runs an in-place one-rank
        # SUM as no work at all, where AVG launches its premultiply kernel over the whole buffer (66 us
        # for the Lego gradient, r4e timeline) -- the one-rank rehearsal then times the data-parallel
        # step's own kernels, not a copy no real run makes
        self._mean_op = NCCL_SUM if self.world == 1 else NCCL_AVG

    @staticmethod
    def _stream():
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def reduce_scatter_avg_(self, shard, flat):
        """shard <- this rank's slice of the mean over ranks of flat (shard may be that slice of flat)."""
        assert flat.numel() == shard.numel() * self.world and flat.dtype == shard.dtype
        _check(_lib().ncclReduceScatter(ctypes.c_void_p(flat.data_ptr()), ctypes.c_void_p(shard.data_ptr()),
                                        shard.numel(), _dtype(shard), self._mean_op, self.comm, self._stream()),
               "ncclReduceScatter")
        return shard

    def all_gather_(self, full):
        """full = concat over ranks of each rank's slice full[rank*k:(rank+1)*k] (in place)."""
        k = full.numel() // self.world
        src = full[self.rank * k:(self.rank + 1) * k]
        _check(_lib().ncclAllGather(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(full.data_ptr()), k, _dtype(full),
                                    self.comm, self._stream()), "ncclAllGather")
        return full

    def all_reduce_avg_(self, flat):
        _check(_lib().ncclAllReduce(ctypes.c_void_p(flat.data_ptr()), ctypes.c_void_p(flat.data_ptr()), flat.numel(),
                                    _dtype(flat), self._mean_op, self.comm, self._stream()), "ncclAllReduce")
        return flat

    def close(self):
        if self.comm:
            _lib().ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()

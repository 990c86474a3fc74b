"""Data parallelism of the training step: every rank holds the fp16 compute copy
of the whole model (table, MLPs) and the occupancy grid, marches its OWN rays (rank-distinct seeds
-- the reference's DDP ranks draw identical batches, base.py:22-33 + seed_everything), and
exchanges per step either
  * ONE all-reduce (mean) of the flat fp32 gradient, then the full Adam on every rank
    (allreduce_mean_), or
  * (default for world > 1, TrainStep.shard_optimizer) a reduce-scatter (mean) of the gradient,
    Adam on this rank's 1/world shard of the fp32 master/m/v only, and an all-gather of the fp16
    compute copy (sharded_update): 1.5 instead of 2 gradient-sized transfers per rank and 1/world
    of the optimizer's HBM traffic; the fp32 master copy stays sharded.
There is no per-step buffer broadcast (DDP's broadcast_buffers moved ~40 MiB/step in the
reference); the occupancy grid is refreshed identically on every rank from identical parameters.
Backend "nccl" is RCCL over xGMI on MI355X; "gloo" is used for the CPU tests.
"""
import os

import torch
import torch.distributed as dist


def rank_seed(base, rank):
    """Seed of rank `rank`'s ray batches (distinct per rank, reproducible)."""
    return int(base) + 1000 * int(rank)


def _host_staged(fn, *ts):
    """gloo has no GPU collectives: run fn on host copies of CUDA tensors and copy results back
    (CPU tests and single-GPU rehearsals only; RCCL takes device tensors directly)."""
    if dist.get_backend() == "nccl" or not any(t.is_cuda for t in ts):
        return fn(*ts)
    hs = [t.cpu() for t in ts]
    fn(*hs)
    for t, h in zip(ts, hs):
        t.copy_(h)


# A one-rank process group skips the collectives (they are identities there, and gloo would copy the
# whole flat gradient and fp16 copy through host memory and back every step) unless a rehearsal asks
# for them: bench.py --dp-rehearse and the one-GPU tests run the backend's single-rank path on purpose.
_REHEARSE = os.environ.get("MFNERF_DP_REHEARSE", "0") == "1"


# the direct RCCL communicator (mfnerf.rccl.Comm), when the backend is RCCL: collectives issued on the
# caller's stream, hence capturable inside the step's HIP graph (TrainStep.capture: "dp_step")
_COMM = None


def use_direct_rccl(on=True):
    """Route the exchange through a direct RCCL communicator (backend "nccl" only; a no-op
    otherwise).  Returns whether it is in use."""
    global _COMM
    if not on:
        if _COMM is not None:
            _COMM.close()
        _COMM = None
        return False
    if _COMM is None and _on() and dist.get_backend() == "nccl":
        from .rccl import Comm
        try:
            _COMM = Comm()
            import atexit
            atexit.register(use_direct_rccl, False)  # ncclCommDestroy at exit (a no-op once closed)
        except (OSError, RuntimeError) as e:  # e.g. no RCCL symbols: keep torch.distributed's collectives
            import warnings
            warnings.warn(f"direct RCCL communicator unavailable ({e}); using torch.distributed collectives")
            _COMM = None
    return _COMM is not None


def direct_rccl():
    """The direct communicator in use (or None)."""
    return _COMM if _on() else None


def rehearse(on=True):
    """Route the collectives through the backend even at world size 1 (measurement / tests)."""
    global _REHEARSE
    _REHEARSE = bool(on)


def _on():
    """A process group of more than one rank is up (or a one-rank group under rehearse())."""
    return dist.is_available() and dist.is_initialized() and (_REHEARSE or dist.get_world_size() > 1)


def allreduce_mean_(flat):
    """In-place mean over ranks of one flat gradient tensor (one collective per step)."""
    if not _on():
        return flat
    if _COMM is not None:
        return _COMM.all_reduce_avg_(flat)
    if dist.get_backend() == "nccl":
        dist.all_reduce(flat, op=dist.ReduceOp.AVG)
    else:
        def f(x):
            dist.all_reduce(x, op=dist.ReduceOp.SUM)
            x.div_(dist.get_world_size())
        _host_staged(f, flat)
    return flat


def _world():
    if not _on():
        return 1
    return dist.get_world_size()


def reduce_scatter_mean_(shard, flat):
    """shard (flat.numel()/world,) <- this rank's slice of the mean over ranks of flat.  shard may be
    flat's own slice [rank*k, (rank+1)*k) (in place: RCCL reduces into it where it lies, no copy)."""
    if not _on():
        if shard.data_ptr() != flat.data_ptr() + _rank() * shard.numel() * shard.element_size():
            shard.copy_(flat[:shard.numel()])
        return shard
    if _COMM is not None:
        return _COMM.reduce_scatter_avg_(shard, flat)
    if dist.get_backend() == "nccl":
        dist.reduce_scatter_tensor(shard, flat, op=dist.ReduceOp.AVG)
    else:
        # host-staged: only the shard is written back (it may alias flat)
        hx = flat.cpu() if flat.is_cuda else flat.clone()
        hs = torch.empty(shard.shape, dtype=shard.dtype)
        dist.reduce_scatter_tensor(hs, hx, op=dist.ReduceOp.SUM)
        hs.div_(dist.get_world_size())
        shard.copy_(hs)
    return shard


def _rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def all_gather_(full, rank):
    """full = concat over ranks of each rank's slice full[rank*k:(rank+1)*k] (in place)."""
    if not _on():
        return full
    if _COMM is not None:
        return _COMM.all_gather_(full)
    w = _world()
    k = full.numel() // w
    if dist.get_backend() == "nccl":  # in place: RCCL reads this rank's slice where it lies
        dist.all_gather_into_tensor(full, full[rank * k:(rank + 1) * k])
    else:
        _host_staged(lambda x: dist.all_gather_into_tensor(x, x[rank * k:(rank + 1) * k].clone()), full)
    return full


def sharded_update(grads, g_shard, p16, rank, adam_shard, flag=None):
    """One ZeRO-1 optimizer step: reduce-scatter(mean) grads into g_shard, adam_shard(g_shard)
    updates this rank's fp32 master / m / v shard and writes its fp16 slice of p16, then the fp16
    slices are all-gathered so every rank holds the full updated compute copy.
    flag (optional device i32[1], this rank's non-finite flag): carried through the reduce-scatter
    (NaN in every shard's first element when set; read back from this rank's shard), so every rank
    sees the union of the flags without another collective."""
    from ._lib import call, ptr, stream
    w = _world()
    if flag is not None and _on():
        call("mfnerf_flag_to_shards", ptr(grads), w, g_shard.numel(), ptr(flag), stream())
    reduce_scatter_mean_(g_shard, grads)
    if flag is not None and _on():
        call("mfnerf_flag_from_shard", ptr(g_shard), ptr(flag), stream())
    adam_shard(g_shard)
    all_gather_(p16, rank)


def allreduce_max_(t):
    """In-place elementwise max over ranks (the non-finite-gradient flag)."""
    if not _on():
        return t
    if dist.get_backend() == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    else:
        _host_staged(lambda x: dist.all_reduce(x, op=dist.ReduceOp.MAX), t)
    return t


def max_over_ranks(x: float, device=None):
    """Slowest rank's value (bench timing)."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t)

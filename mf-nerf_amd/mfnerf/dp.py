"""Data parallelism of the training step: every rank holds a full replica (table,
MLPs, occupancy), marches its OWN rays (rank-distinct seeds -- the reference's DDP ranks draw
identical batches, base.py:22-33 + seed_everything), and the only exchange per step is ONE
all-reduce (mean) of the flat fp32 gradient vector between backward and Adam.  There is no
per-step buffer broadcast (DDP's broadcast_buffers moved ~40 MiB/step in the reference); the
occupancy grid is refreshed identically on every rank from identical parameters.
Backend "nccl" is RCCL over xGMI on MI355X; "gloo" is used for the CPU tests.
"""
import torch
import torch.distributed as dist


def rank_seed(base, rank):
    """Seed of rank `rank`'s ray batches (distinct per rank, reproducible)."""
    return int(base) + 1000 * int(rank)


def allreduce_mean_(flat):
    """In-place mean over ranks of one flat gradient tensor (one collective per step)."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return flat
    if dist.get_backend() == "nccl":
        dist.all_reduce(flat, op=dist.ReduceOp.AVG)
    else:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat.div_(dist.get_world_size())
    return flat


def max_over_ranks(x: float, device=None):
    """Slowest rank's value (bench timing)."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t)

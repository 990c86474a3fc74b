"""world_size=2 data-parallel step semantics on CPU over gloo: rank-distinct batches, one mean
all-reduce of the flat gradient, identical Adam updates -> bitwise-identical replicas."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def adam_ref(p, g, m, v, t, lr=1e-2, b1=0.9, b2=0.999, eps=1e-15):
    """The update of mfnerf_adam_step (apex FusedAdam, decay 0)."""
    m.mul_(b1).add_((1 - b1) * g)
    v.mul_(b2).add_((1 - b2) * g * g)
    p.sub_(lr * ((m / (1 - b1 ** t)) / (torch.sqrt(v / (1 - b2 ** t)) + eps)))


def _worker(rank, world, port, out):
    import sys
    sys.path[:0] = [ROOT, PKG]
    from mfnerf import dp
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)  # identical init on every rank
    p = torch.randn(1000)
    m, v = torch.zeros(1000), torch.zeros(1000)
    for t in range(1, 4):
        g = torch.Generator().manual_seed(dp.rank_seed(t, rank))  # rank-distinct "batch"
        grad = torch.randn(1000, generator=g)
        local = grad.clone()
        dp.allreduce_mean_(grad)
        gathered = [torch.zeros(1000) for _ in range(world)]
        dist.all_gather(gathered, local)
        assert torch.allclose(grad, torch.stack(gathered).mean(0), atol=1e-6)
        assert not torch.equal(gathered[0], gathered[1])
        adam_ref(p, grad, m, v, t)
    out[rank] = p
    assert dp.max_over_ranks(float(rank)) == world - 1
    dist.destroy_process_group()


def test_two_rank_step_keeps_replicas_identical():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert torch.equal(out[0], out[1])


def _sharded_worker(rank, world, port, out):
    import sys
    sys.path[:0] = [ROOT, PKG]
    from mfnerf import dp
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1024  # padded flat parameter vector
    torch.manual_seed(0)
    p_full = torch.randn(n)
    p_full[1000:] = 0.0  # padding: zero, zero grads -> stays zero
    k = n // world
    lo, hi = rank * k, (rank + 1) * k
    # replica A: all-reduce + full Adam; replica B: sharded (this rank's fp32 master/m/v slice only)
    pa, ma, va = p_full.clone(), torch.zeros(n), torch.zeros(n)
    pb, mb, vb = p_full.clone(), torch.zeros(k), torch.zeros(k)
    p16 = p_full.half()
    g_shard = torch.zeros(k)
    for t in range(1, 5):
        g = torch.Generator().manual_seed(dp.rank_seed(t, rank))
        grad = torch.randn(n, generator=g)
        grad[1000:] = 0.0
        ga = dp.allreduce_mean_(grad.clone())
        adam_ref(pa, ga, ma, va, t)

        def adam_shard(gs):
            adam_ref(pb[lo:hi], gs, mb, vb, t)
            p16[lo:hi] = pb[lo:hi].half()

        dp.sharded_update(grad.clone(), g_shard, p16, rank, adam_shard)
        # the fp16 compute copy every rank holds equals the all-reduce replica's, bit for bit
        assert torch.equal(p16, pa.half()), t
        assert torch.equal(pb[lo:hi], pa[lo:hi])
    assert torch.equal(p16[1000:], torch.zeros(n - 1000, dtype=torch.float16))
    out[rank] = p16
    dist.destroy_process_group()


def test_two_rank_sharded_optimizer_matches_allreduce():
    """ZeRO-1 update (reduce-scatter mean -> Adam on the shard -> all-gather fp16) == all-reduce
    mean -> full Adam, bit for bit, and leaves identical compute copies on every rank."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_sharded_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert torch.equal(out[0], out[1])


class _Counting:
    """Counts the process-group collectives a callable issues (torch.distributed patched)."""

    def __init__(self):
        self.n = 0

    def __enter__(self):
        self._saved = {k: getattr(dist, k) for k in ("all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor")}
        for k, f in self._saved.items():
            def wrap(*a, _f=f, **kw):
                self.n += 1
                return _f(*a, **kw)
            setattr(dist, k, wrap)
        return self

    def __exit__(self, *exc):
        for k, f in self._saved.items():
            setattr(dist, k, f)


def _one_rank_worker(rank, port, out):
    import sys
    sys.path[:0] = [ROOT, PKG]
    from mfnerf import dp
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    x = torch.randn(4096)
    sh, full = torch.empty(4096), x.half()
    res = []
    for rehearse in (False, True):
        dp.rehearse(rehearse)
        with _Counting() as c:
            y = dp.allreduce_mean_(x.clone())
            dp.reduce_scatter_mean_(sh, x)
            dp.all_gather_(full, 0)
        res.append((c.n, torch.equal(y, x), torch.equal(sh, x), torch.equal(full, x.half())))
    dp.rehearse(False)
    # the direct RCCL communicator (captured collectives) exists only over an RCCL process group
    dp.rehearse(True)
    res.append(dp.use_direct_rccl())
    dp.rehearse(False)
    out["r"] = res
    dist.destroy_process_group()


def test_one_rank_group_skips_collectives_unless_rehearsing():
    """A one-rank process group pays nothing per step (the collectives are identities and gloo would
    stage the flat gradient through host memory); dp.rehearse() routes them through the backend."""
    out = mp.Manager().dict()
    mp.spawn(_one_rank_worker, args=(_free_port(), out), nprocs=1, join=True)
    (n_off, *ok_off), (n_on, *ok_on), direct = out["r"]
    assert direct is False
    assert n_off == 0 and all(ok_off)
    assert n_on == 3 and all(ok_on)

"""Data parallel on ONE GPU (gloo, host-staged collectives, 2 processes sharing cuda:0): the real
engine's exchange paths.  RCCL needs one GPU per rank and is exercised by the multi-GPU bench."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mfnerf import dp, engine, synthetic
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    st = engine.TrainStep(engine.StepConfig(n_rays=512, log2_T=14), device=dev, seed=0)
    st.set_occupancy(synthetic.ball_density_grid())
    if mode == "shard":
        st.shard_optimizer(rank, world)
    ex = dp.allreduce_mean_ if mode == "allreduce" else None
    good = st.make_batches(2, seed=dp.rank_seed(100, rank))
    st.run(good[0], exchange=ex)
    p1, s1 = st.p16.clone(), int(st.step_dev)
    bad = st.make_batches(1, seed=dp.rank_seed(200, rank))[0]
    if rank == 1:
        bad.rgb.fill_(float("nan"))  # only rank 1's gradient is non-finite
    st.run(bad, exchange=ex)
    torch.cuda.synchronize()
    skipped = (torch.equal(st.p16, p1), int(st.step_dev) == s1, st.skipped_steps())
    st.run(good[1], exchange=ex)
    torch.cuda.synchronize()
    out[(mode, rank)] = (skipped, st.p16.cpu(), bool(torch.isfinite(st.p16).all()), int(st.step_dev))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["shard", "allreduce"])
def test_nonfinite_on_one_rank_skips_on_every_rank(mode):
    """GradScaler semantics across ranks: a NaN in ONE rank's gradient skips the step on ALL ranks
    (the flag rides the reduce-scatter / all-reduce), replicas stay identical and finite, and the
    next clean step updates everywhere."""
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _port(), mode, out), nprocs=world, join=True)
    for r in range(world):
        skipped, p16, finite, steps = out[(mode, r)]
        assert skipped == (True, True, 1), (r, skipped)
        assert finite and steps == 2
        assert torch.equal(p16, out[(mode, 0)][1])


def _replay_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mfnerf import dp, engine, synthetic
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    st = engine.TrainStep(engine.StepConfig(n_rays=512, log2_T=14), device=dev, seed=0)
    st.set_occupancy(synthetic.ball_density_grid())
    st.shard_optimizer(rank, world)
    good = st.make_batches(3, seed=dp.rank_seed(100, rank))
    bad = st.make_batches(1, seed=dp.rank_seed(200, rank))[0]
    if rank == 1:
        bad.rgb.fill_(float("nan"))
    g = torch.Generator().manual_seed(rank + 5)
    noise = [torch.rand(512, generator=g).to(dev) for _ in range(4)]
    st.run(good[0], noise=noise[0])
    st.capture(host_noise=True)
    st.replay(good[1], noise=noise[1], next_batch=bad, next_noise=noise[2])
    torch.cuda.synchronize()
    p1, s1, l1 = st.p16.clone(), int(st.step_dev), st._level_l1.clone()
    st.replay(bad, noise=noise[2], next_batch=good[2], next_noise=noise[3])
    torch.cuda.synchronize()
    skipped = (torch.equal(st.p16, p1), int(st.step_dev) == s1, st.skipped_steps(),
               int(torch.count_nonzero(st._level_l1)), int(torch.count_nonzero(l1)))
    st.replay(good[2], noise=noise[3])
    torch.cuda.synchronize()
    out[rank] = (skipped, st.p16.cpu(), bool(torch.isfinite(st.p16).all()), int(st.step_dev))
    dist.destroy_process_group()


def test_nonfinite_on_one_rank_skips_replayed_sharded_step():
    """The same through the captured sharded step (dp_pre / reduce-scatter / dp_post graphs): the
    update reads the exchanged flag from its shard in the Adam launch itself
    (mfnerf_adam_step_shard), skips on every rank, and leaves the level L1 bounds zeroed either way."""
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_replay_worker, args=(world, _port(), out), nprocs=world, join=True)
    for r in range(world):
        skipped, p16, finite, steps = out[r]
        assert skipped == (True, True, 1, 0, 0), (r, skipped)
        assert finite and steps == 3
        assert torch.equal(p16, out[0][1])


def _union_worker(rank, world, port, mode, out):
    """Rank r trains on its half of a 2N-ray batch; the exchange must make every rank's step equal
    to ONE process stepping on the union (the reference's DDP semantics: mean of the ranks' mean
    gradients = gradient of the mean loss over all rays)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mfnerf import dp, engine, synthetic
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n = 512
    st = engine.TrainStep(engine.StepConfig(n_rays=n, log2_T=14), device=dev, seed=0)
    st.set_occupancy(synthetic.ball_density_grid())
    full = _union_batch(2 * n, dev)
    mine = engine.Batch(*(t[rank * n:(rank + 1) * n].contiguous() for t in (full.rays_o, full.rays_d, full.rgb)))
    noise = _union_noise(2 * n)[rank * n:(rank + 1) * n].to(dev)
    # 1) the exchanged gradient (the all-reduce's mean) of one step, before Adam
    st.run(mine, optimize=False, noise=noise)
    g = st.grads.clone()
    dp.allreduce_mean_(g)
    # 2) a whole step through the mode's exchange + optimizer
    st2 = engine.TrainStep(engine.StepConfig(n_rays=n, log2_T=14), device=dev, seed=0)
    st2.set_occupancy(synthetic.ball_density_grid())
    if mode == "shard":
        st2.shard_optimizer(rank, world)
    st2.run(mine, exchange=dp.allreduce_mean_ if mode == "allreduce" else None, noise=noise)
    torch.cuda.synchronize()
    out[(mode, rank)] = (g.cpu(), st2.full_params().cpu(), st2.p16.cpu(), int(st2.step_dev))
    dist.destroy_process_group()


def _union_batch(n2, dev):
    from mfnerf import engine
    st = engine.TrainStep(engine.StepConfig(n_rays=n2, log2_T=14), device=dev, seed=0)
    b = st.make_batches(1, seed=300)[0]
    return engine.Batch(b.rays_o.contiguous(), b.rays_d.contiguous(), b.rgb.contiguous())


def _union_noise(n2):
    return torch.rand(n2, generator=torch.Generator().manual_seed(77))


@pytest.mark.parametrize("mode", ["shard", "allreduce"])
def test_two_ranks_equal_one_process_on_the_union_batch(gpu, mode):
    """world 2 (gloo, both ranks on cuda:0), batches A and B vs one process on A u B (2N rays),
    same initial weights, occupancy and march perturbations:
      * the exchanged gradient equals the single process's gradient -- MLP blocks to fp16-backward
        reassociation (sums over different sample sets), table regions to the fixed-point resolution
        (each rank rounds to its own per-level quantum): max 5e-4 of a region's largest entry, 1e-4 of
        its L2 norm;
      * after the mode's exchange + Adam, the parameters agree wherever the gradient is not at the
        resolution floor (Adam with eps 1e-15 turns any non-zero gradient into a ~lr step, so entries
        whose gradient is ~1e-6 of the largest may legitimately move differently), replicas are
        identical on both ranks, and the step counter advanced once."""
    from mfnerf import engine, synthetic
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_union_worker, args=(world, _port(), mode, out), nprocs=world, join=True)
    n = 512
    st = engine.TrainStep(engine.StepConfig(n_rays=2 * n, log2_T=14), device=gpu, seed=0)
    st.set_occupancy(synthetic.ball_density_grid())
    full = _union_batch(2 * n, gpu)
    noise = _union_noise(2 * n).to(gpu)
    st.run(full, optimize=False, noise=noise)
    gu = st.grads.cpu()
    g0, p0, h0, s0 = out[(mode, 0)]
    g1, p1, h1, s1 = out[(mode, 1)]
    assert torch.equal(g0, g1) and torch.equal(h0, h1) and torch.equal(p0, p1)  # identical replicas
    assert s0 == s1 == 1
    lay = st.layout
    cuts = [0, engine.XYZ_NET_PARAMS, st.off_table] + [st.off_table + 2 * o for o in sorted(set(lay.offsets))[1:]] \
        + [st.n_params]
    for a, b in zip(cuts[:-1], cuts[1:]):
        scale = float(gu[a:b].abs().max())
        if scale > 0:
            # each rank rounds its run-merged contributions to its own quantum 2^-30 x (its level L1):
            # a few quanta per entry, ~1e-4 of a region's largest entry for the densest (coarse) levels
            d = g0[a:b] - gu[a:b]
            assert float(d.abs().max()) <= 5e-4 * scale, (mode, a, b, float(d.abs().max()) / scale)
            assert float(d.norm()) <= 1e-4 * float(gu[a:b].norm()), (mode, a, b)
    # a whole step on the union in one process
    st2 = engine.TrainStep(engine.StepConfig(n_rays=2 * n, log2_T=14), device=gpu, seed=0)
    st2.set_occupancy(synthetic.ball_density_grid())
    st2.run(full, noise=noise)
    pu = st2.params[:st.n_params].cpu()
    pd = p0[:st.n_params]
    moved = (pd - pu).abs()
    floor = gu[:st.n_params].abs() <= 1e-6 * float(gu[:st.n_params].abs().max())
    assert float(moved[~floor].max()) <= 1e-5, (mode, float(moved[~floor].max()))
    assert float(moved.max()) <= 2.1 * st.cfg.lr  # at most one opposite ~lr step at the floor

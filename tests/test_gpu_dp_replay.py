"""The data-parallel step as bench.py --gpus N runs it (config 5: ray-sharded DDP, train.py:277-287),
on the one-GPU box:

* two gloo ranks sharing cuda:0, each with its own rank-seeded DeviceDataset, capture() + replay()
  exactly as bench.py's timed loop drives them (one-graph-per-side DP path: dp_pre -> collective ->
  dp_post, the next march gated; one step through the per-stage graphs as bench's event-timed steps
  take), against the eager DP step on the same ranks -- both exchange modes;
* the same two ranks on explicit halves of a batch over several replayed steps against ONE process
  stepping on the union (the reference's DDP semantics: the mean of the ranks' mean gradients is the
  gradient of the mean loss);
* a one-rank RCCL ("nccl") process group: reduce-scatter / all-gather / all-reduce through their RCCL
  branches (eager and replayed), bit-identical to the single-process step.
Ranks share the GPU over host-staged gloo collectives; RCCL across GPUs runs in the driver's
multi-GPU bench."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_RAYS, LOG2_T = 1024, 15


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dataset(rank, dev):
    """bench.py's data: analytic views of the calibrated ball scene, rank-distinct draws."""
    from mfnerf import data, dp, synthetic
    scene = data.BallScene.matching_grid(seed=0)
    imgs, poses, dirs, K = data.ball_scene_views(scene, 8, 64, synthetic.LEGO_F * 64 / synthetic.LEGO_W,
                                                 seed=dp.rank_seed(100, rank), device=dev)
    return data.DeviceDataset(imgs, poses, dirs, K=K, img_wh=(64, 64), device=dev, seed=dp.rank_seed(7, rank))


def _step(dev, mode, rank, world, ds=None, n_rays=N_RAYS):
    from mfnerf import engine, synthetic
    st = engine.TrainStep(engine.StepConfig(n_rays=n_rays, log2_T=LOG2_T), device=dev, seed=0)
    st.set_occupancy(synthetic.ball_density_grid())
    if mode == "shard":
        st.shard_optimizer(rank, world, force=True)
    if ds is not None:
        st.attach_dataset(ds)
    return st


def _state(st):
    return {"params": st.full_params().cpu(), "p16": st.p16.cpu(), "packed": st.packed.cpu(),
            "steps": int(st.step_dev), "loss": float(st.loss_sum)}


def _bench_worker(rank, world, port, mode, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mfnerf import dp
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    ex = dp.allreduce_mean_ if mode == "allreduce" else None
    K = 5
    xb = _batches(1, N_RAYS, dev)[0]  # an explicit batch for the eager step after the replays
    xn = torch.rand(N_RAYS, generator=torch.Generator().manual_seed(rank + 11)).to(dev)

    def replayed():
        # as bench.py: eager warm-up step, capture, replays (step 2 event-timed: per-stage graphs);
        # the last one-graph replay defers its MLP repack to the next step's graph
        a = _step(dev, mode, rank, world, _dataset(rank, dev))
        a.run(exchange=ex)
        a.capture()
        mk = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
        for k in range(1, K):
            a.replay(exchange=ex, grid_bw_events=(mk(), [mk()]) if k == 2 else None)
        return a

    def eager():
        b = _step(dev, mode, rank, world, _dataset(rank, dev))
        for k in range(K):
            b.run(exchange=ex)
        return b

    res = {}
    # (1) an eager step right after the replays (it must repack first)
    a, b = replayed(), eager()
    a.run(xb, exchange=ex, noise=xn)
    b.run(xb, exchange=ex, noise=xn)
    torch.cuda.synchronize()
    res["run"] = (_state(a), _state(b))
    # (2) an occupancy refresh right after the replays: its density query runs the field on the
    # packed weights, so the refreshed grid shows whether they were current
    a, b = replayed(), eager()
    a.update_density_grid()
    b.update_density_grid()
    torch.cuda.synchronize()
    sa, sb = _state(a), _state(b)
    sa["grid"], sb["grid"] = a.density_grid.cpu(), b.density_grid.cpu()
    res["refresh"] = (sa, sb)
    out[(mode, rank)] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["shard", "allreduce"])
def test_dp_replay_as_bench_matches_eager_dp(mode):
    """bench.py's replay path (dp_pre / collective / dp_post graphs, gated march, one event-timed
    per-stage step in between), then an occupancy refresh and an eager step, leaves every rank
    bit-identical to the eager DP steps on the same batches (weights, fp16 copy, packed MLP blob,
    density grid), and the replicas identical across ranks."""
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_bench_worker, args=(world, _port(), mode, out), nprocs=world, join=True)
    for r in range(world):
        for case, (got, ref) in out[(mode, r)].items():
            assert got["steps"] == ref["steps"] == (6 if case == "run" else 5), (case, got["steps"], ref["steps"])
            for key in ("params", "p16", "packed") + (("grid",) if case == "refresh" else ()):
                assert torch.equal(got[key], ref[key]), (mode, r, case, key,
                                                         float((got[key].float() - ref[key].float()).abs().max()))
            assert torch.isfinite(got["params"]).all()
            g0 = out[(mode, 0)][case][0]
            assert torch.equal(got["params"], g0["params"]) and torch.equal(got["p16"], g0["p16"])


def _batches(k, n2, dev):
    from mfnerf import engine
    st = engine.TrainStep(engine.StepConfig(n_rays=n2, log2_T=LOG2_T), device=dev, seed=0)
    return [engine.Batch(b.rays_o.contiguous(), b.rays_d.contiguous(), b.rgb.contiguous())
            for b in st.make_batches(k, seed=300)]


def _noises(k, n2):
    g = torch.Generator().manual_seed(77)
    return [torch.rand(n2, generator=g) for _ in range(k)]


def _half(b, rank, n):
    from mfnerf import engine
    return engine.Batch(*(t[rank * n:(rank + 1) * n].contiguous() for t in (b.rays_o, b.rays_d, b.rgb)))


def _union_worker(rank, world, port, mode, K, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mfnerf import dp
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n = N_RAYS
    full = _batches(K + 1, 2 * n, dev)
    noise = [z[rank * n:(rank + 1) * n].to(dev) for z in _noises(K + 1, 2 * n)]
    mine = [_half(b, rank, n) for b in full]
    ex = dp.allreduce_mean_ if mode == "allreduce" else None
    st = _step(dev, mode, rank, world)
    st.run(mine[0], exchange=ex, noise=noise[0])
    losses = [float(st.loss_sum)]
    st.capture(host_noise=True)
    for k in range(1, K):
        nxt = k + 1 < K
        st.replay(mine[k], exchange=ex, noise=noise[k], next_batch=mine[k + 1] if nxt else None,
                  next_noise=noise[k + 1] if nxt else None)
        losses.append(float(st.loss_sum))
    torch.cuda.synchronize()
    out[(mode, rank)] = (st.full_params().cpu(), st.p16.cpu(), int(st.step_dev), losses)
    dist.destroy_process_group()


def _union_single(gpu, K, n2, parts):
    """One process stepping eagerly on the union batches (parts: 2 = float table-gradient atomics and
    other summation orders -- an equally valid implementation of the same step).  Returns the final
    parameters and the per-step losses."""
    from mfnerf import engine, synthetic
    full = _batches(K + 1, n2, gpu)
    noise = _noises(K + 1, n2)
    st = engine.TrainStep(engine.StepConfig(n_rays=n2, log2_T=LOG2_T, n_parts=parts), device=gpu, seed=0)
    st.set_occupancy(synthetic.ball_density_grid())
    losses = []
    for k in range(K):
        st.run(full[k], noise=noise[k].to(gpu))
        losses.append(float(st.loss_sum))
    torch.cuda.synchronize()
    return st, st.params[:st.n_params].cpu(), losses


@pytest.mark.parametrize("mode", ["shard", "allreduce"])
def test_replayed_ranks_equal_one_process_on_the_union_batch(gpu, mode):
    """Two ranks replaying K = 4 steps on halves A_k, B_k vs one process stepping eagerly on
    A_k u B_k (2N rays), same initial weights, occupancy and march perturbations.  Each step's loss
    is the mean of the ranks' losses.  The parameters cannot agree bit for bit (the ranks round their
    table-gradient contributions at their own fixed-point quanta, and Adam with eps 1e-15 turns any
    sign flip of a near-zero gradient into a ~lr step, which the next steps propagate), so they are
    held to the divergence between two equally valid single-process implementations of the union
    step: the same batches through 2 ray parts (float table-gradient atomics, other MLP summation
    order).  Per block (MLPs, table), the data-parallel run's L2 distance to the one-part run must
    stay within 3x that natural distance.  Replicas are identical."""
    world, K, n = 2, 4, N_RAYS
    out = mp.Manager().dict()
    mp.spawn(_union_worker, args=(world, _port(), mode, K, out), nprocs=world, join=True)
    p0, h0, s0, l0 = out[(mode, 0)]
    p1, h1, s1, l1 = out[(mode, 1)]
    assert torch.equal(p0, p1) and torch.equal(h0, h1) and s0 == s1 == K
    st, pu, lu = _union_single(gpu, K, 2 * n, 1)
    _, pv, lv = _union_single(gpu, K, 2 * n, 2)
    for k in range(K):
        assert abs((l0[k] + l1[k]) / 2 - lu[k]) <= 2e-3 * abs(lu[k]), (mode, k, l0[k], l1[k], lu[k])
    pd = p0[:st.n_params]
    for name, a, b in (("mlp", 0, st.off_table), ("table", st.off_table, st.n_params)):
        d_dp = float((pd[a:b] - pu[a:b]).norm())
        d_nat = float((pv[a:b] - pu[a:b]).norm())
        print(f"\nUNION {mode} {name}: |dp - union| {d_dp:.4g}, |union 2 parts - union| {d_nat:.4g}, "
              f"|union| {float(pu[a:b].norm()):.4g}")
        assert d_dp <= 3.0 * d_nat + 1e-6 * float(pu[a:b].norm()), (mode, name, d_dp, d_nat)


def _nccl_worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from mfnerf import dp
    dp.rehearse(True)  # a one-rank group skips its collectives unless rehearsing
    assert dist.get_backend() == "nccl"
    # the collectives' RCCL branches on device tensors
    x = torch.randn(4096, device=dev)
    y = x.clone()
    dp.allreduce_mean_(y)
    sh = torch.empty(4096, device=dev)
    dp.reduce_scatter_mean_(sh, x)
    z = x.half()
    dp.all_gather_(z, 0)
    m = torch.tensor([3.0], device=dev)
    dp.allreduce_max_(m)
    torch.cuda.synchronize()
    prims = (torch.equal(y, x), torch.equal(sh, x), torch.equal(z, x.half()), float(m) == 3.0)
    res = {}
    for direct in (False, True):
        # torch.distributed's RCCL collectives between two graphs, then the direct communicator
        # (mfnerf/rccl.py) whose collectives are captured: the step as one graph ("dp_step")
        assert dp.use_direct_rccl(direct) == direct
        for mode in ("shard", "allreduce"):
            ex = dp.allreduce_mean_ if mode == "allreduce" else None
            a = _step(dev, mode, 0, 1, _dataset(0, dev))
            for _ in range(2):
                a.run(exchange=ex)                     # eager: sharded_update / all-reduce over RCCL
            a.capture()
            assert (a.graphs.get("dp_step") is not None) == direct
            for _ in range(3):
                a.replay(exchange=ex)                  # dp_pre -> RCCL -> dp_post, or dp_step
            torch.cuda.synchronize()
            res[(mode, direct)] = _state(a)
    dp.use_direct_rccl(False)
    ref = _step(dev, "none", 0, 1, _dataset(0, dev))  # no process group involved in its step
    for _ in range(5):
        ref.run()
    torch.cuda.synchronize()
    out["r"] = (prims, res, _state(ref))
    dist.destroy_process_group()


def test_rccl_one_rank_matches_single_process():
    """init_process_group('nccl') at world size 1 on the one GPU: allreduce_mean_, reduce_scatter_mean_,
    all_gather_ and allreduce_max_ take their RCCL branches (identity at one rank); two eager and
    three replayed DP steps in both modes, through torch.distributed and through the direct RCCL
    communicator captured in the step graph, leave the parameters bit-identical to five plain
    single-process steps on the same draws."""
    out = mp.Manager().dict()
    mp.spawn(_nccl_worker, args=(_port(), out), nprocs=1, join=True)
    prims, res, ref = out["r"]
    assert all(prims), prims
    for mode, got in res.items():
        assert got["steps"] == ref["steps"] == 5, mode
        for key in ("params", "p16"):
            assert torch.equal(got[key], ref[key]), (mode, key, float((got[key].float() - ref[key].float()).abs().max()))

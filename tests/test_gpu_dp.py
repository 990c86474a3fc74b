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

"""Rehearse the data-parallel training step on ONE GPU: `world` processes share cuda:0 over gloo
(host-staged collectives), each running the real engine (HIP kernels, graphs) with rank-distinct
rays.  Checks: every rank ends with the identical fp16 compute copy, and the sharded optimizer and
the all-reduce path give bit-identical compute copies.  (RCCL itself needs one GPU per rank; the
driver's multi-GPU bench exercises it.)  Usage: python tools/dp_rehearsal.py [world]"""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def worker(rank, world, port, mode, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mfnerf import dp, engine, synthetic
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    st = engine.TrainStep(engine.StepConfig(n_rays=2048, log2_T=16), device=dev, seed=0)
    st.set_occupancy(synthetic.ball_density_grid())
    if mode == "shard":
        st.shard_optimizer(rank, world)
    ex = dp.allreduce_mean_ if mode == "allreduce" else None
    bs = st.make_batches(6, seed=dp.rank_seed(100, rank))
    st.run(bs[0], exchange=ex)              # eager step (lazy init)
    st.capture()
    for k in range(1, 5):                    # pipelined graph replays
        st.replay(bs[k], exchange=ex, next_batch=bs[k + 1] if k + 1 < 5 else None)
    torch.cuda.synchronize()
    out[(mode, rank)] = st.p16.cpu()
    dist.destroy_process_group()


def port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    mgr = mp.Manager()
    out = mgr.dict()
    for mode in ("shard", "allreduce"):
        mp.spawn(worker, args=(world, port(), mode, out), nprocs=world, join=True)
    for mode in ("shard", "allreduce"):
        for r in range(1, world):
            assert torch.equal(out[(mode, r)], out[(mode, 0)]), f"{mode}: rank {r} replica differs"
    same = torch.equal(out[("shard", 0)], out[("allreduce", 0)])
    diff = (out[("shard", 0)].float() - out[("allreduce", 0)].float()).abs().max().item()
    print(f"world {world}: replicas identical in both modes; shard == allreduce bitwise: {same} (max |diff| {diff:.3g})")
    assert same or diff < 1e-3

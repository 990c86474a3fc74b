"""Training-throughput benchmark of the MF-NeRF hot path on MI355X.

One step = one NeRF training iteration on a synthetic Lego-like batch (BASELINE config 2:
8192 rays/batch per GPU, Hash grid L=16 F=2 T=2^19, rgb 64x2): AABB -> ray march -> grid encode
-> MFMA field head -> composite -> loss -> composite bw -> field bw -> grid bw -> [all-reduce] ->
Adam.  The timed steps replay the step as three HIP graphs (mfnerf.engine.TrainStep.capture);
a preceding eager pass gives the per-kernel breakdown (eager_stage_ms).  The occupancy-grid
refresh (every 16 steps in the reference) is excluded from the timed step as SURVEY.md 8d
prescribes and reported separately (density_update_ms, value_with_occupancy_refresh).

python bench.py [--gpus N --steps K --warmup W]; N>1 runs one rank per GPU (rank-distinct rays,
reduce-scatter of the flat fp32 gradient + sharded Adam + fp16 all-gather per step over RCCL):
either under an outer torch.distributed.run (the driver's launch; WORLD_SIZE must equal N) or, when
started directly, by starting torch.distributed.run itself as a CHILD process before any HIP call
(launch_ranks) and passing rank 0's one JSON line through.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]
# before the HIP runtime initialises (the same default mfnerf/__init__.py sets): graph replays
# through the per-node launch path, ~3 us per step less
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# the table-gradient scatter's kernels in the PMC summaries: the run-merging atomics (dense levels)
# and the partitioned hashed levels' scatter / accumulate
GRID_BW_KERNEL = ("grid_bw_dense_kernel", "grid_bw_kernel", "bin_scatter_kernel", "bin_accum_kernel")
# ... but not the accumulate's fused-Adam instantiation (the graph-replayed steps' launches): the roofline
# times the unfused launches (--roofline-every), whose PMC rows are bin_accum_kernel<false>
GRID_BW_EXCLUDE = ("bin_accum_kernel<true>",)

# algorithmic bytes per live sample of each per-sample kernel, as SURVEY.md 8(d) prices them (the
# tcnn form of the op: fp16 features and fp16 gradient scatter), DESIGN.md section 5
L, F = 16, 2
BYTES_PER_SAMPLE = {
    "grid_fw": 12 + L * 8 * F * 2 + L * F * 2,          # xyz + fp16 corner gathers + fp16 features = 588
    "grid_bw": L * F * 2 + 12 + L * 8 * F * 2,          # fp16 dL/dy + xyz + fp16 scatter of 8 corners = 588
    "field_fw": L * F * 2 + 12 + 4 + 12,                 # feat + dir + sigma + rgb = 92
    "field_bw": L * F * 2 + 12 + 16 + L * F * 4,         # feat + dir + dsigma,drgb + dfeat = 220
}
# measured memory-side int32 atomic request ceiling of MI355X (tools/atomic_probe3.hip)
ATOMIC_REQ_PEAK_G = 26.7


# BASELINE.json configs as step presets.  "lego" (config 2) is the one the metric is quoted on and the
# default; "mf128" is config 3's field (benchmarking/benchmark_synthetic_mf.sh: --grid MixedFeature
# --N_tables 8 --T 20 --batch_size 16384 --lr 2e-2 --rgb_channels 128) on the same synthetic scene.
PRESETS = {
    "lego": dict(n_rays=8192, log2_T=19, grid="Hash", N_tables=1, rgb_width=64, lr=1e-2),
    "mf128": dict(n_rays=16384, log2_T=20, grid="MixedFeature", N_tables=8, rgb_width=128, lr=2e-2),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--preset", choices=sorted(PRESETS), default="lego")
    ap.add_argument("--n-rays", type=int, default=None, help="override the preset's rays per GPU")
    ap.add_argument("--log2-T", type=int, default=None, help="override the preset's log2 table size")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--roofline-every", type=int, default=25,
                    help="time grid_bw with events on every k-th timed step (those steps replay the scatter "
                         "as its own graph, ~45 us more per such step than the one-graph step (r4h: 0.5645 "
                         "ms/step at k = 8 vs 0.5588 at k = 1000); the others replay the whole step as one "
                         "graph); 25: 8 timed launches in the default 200 steps")
    ap.add_argument("--eager", action="store_true", help="time eager launches instead of the HIP graphs")
    ap.add_argument("--parts", type=int, default=1, help="ray-range parts per step (chain/scatter overlap)")
    ap.add_argument("--dp", choices=("shard", "allreduce"), default="shard",
                    help="N>1: sharded optimizer (reduce-scatter + all-gather fp16) or all-reduce + full Adam")
    ap.add_argument("--dp-rehearse", action="store_true",
                    help="N=1: run the N>1 step anyway (a one-rank RCCL group, --dp mode) -- the data-parallel "
                         "path's cost over the single-GPU step with the collectives reduced to a local copy")
    ap.add_argument("--stub-step", action="store_true",
                    help="launcher test only: the rank plumbing, timing and JSON line of a real run around a "
                         "host-only stub step over gloo (no GPU is touched; tests/test_bench_launcher.py)")
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`bench.py --gpus N` (N > 1) started without an outer launcher: run N ranks under
    torch.distributed.run (the driver's own command line: one node, 127.0.0.1) as a CHILD process --
    this process has made no HIP call, and it is never replaced (no exec) -- and pass through exactly
    one JSON line, rank 0's.  Everything else the child writes to stdout goes to stderr.  Returns the
    child's exit status (non-zero as well when the child did not print exactly one line)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC, which RCCL needs on this host driver
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    lines = []
    for line in proc.stdout:
        try:
            rec = json.loads(line)
        except ValueError:
            rec = None
        if isinstance(rec, dict) and "metric" in rec:
            lines.append(line.strip())
        else:
            sys.stderr.write(line)
    rc = proc.wait()
    if len(lines) == 1:
        print(lines[0], flush=True)
    elif rc == 0:
        sys.stderr.write(f"bench.py: expected one JSON line from rank 0, got {len(lines)}\n")
        rc = 1
    return rc


def _marker(ev):
    def mark(name):
        if ev is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ev.append((name, e))
    return mark


def run_step(step, batch, world, ev=None, allreduce=None):
    """One eager training step (mfnerf.engine.TrainStep.run); with ev, an event after every stage."""
    from mfnerf import dp
    mark = _marker(ev)
    mark("start")
    if allreduce is None:
        allreduce = world > 1
    step.run(batch, mark=mark, exchange=dp.allreduce_mean_ if allreduce else None)


def pmc_suffix(preset, log2_T, n_rays):
    """The PMC summary's file suffix for a workload: "" for the lego preset as configured, "_<preset>"
    for another preset, "_T<k>" / "_n<rays>" where the table size / batch differ from the preset's
    (tools/gpu_pmc.sh names its outputs the same way)."""
    pre = PRESETS[preset]
    suffix = "" if preset == "lego" else "_" + preset
    if log2_T is not None and log2_T != pre["log2_T"]:
        suffix += f"_T{log2_T}"
    if n_rays is not None and n_rays != pre["n_rays"]:
        suffix += f"_n{n_rays}"
    return suffix


def pmc_traffic(kernel_prefix, preset="lego", log2_T=None, n_rays=None):
    """(HBM-side bytes, memory-side atomic requests, source) per launch, summed over the kernels whose
    names start with one of `kernel_prefix` (one step's launches of them), from the newest
    committed PMC summary of this workload (profiles/rNN_*pmc_traffic<pmc_suffix>.json, made by
    tools/pmc_traffic.py from separate FETCH_SIZE / WRITE_SIZE / TCC_EA0_ATOMIC rocprofv3 passes with
    the guide's gfx950 corrections); Nones if there is none for this exact workload."""
    import glob
    import re

    def order(f):  # profiles/rNN_vMM_pmc_traffic.json: newest round, then newest version
        m = re.match(r"r(\d+)(?:_v(\d+))?_", os.path.basename(f))
        return (int(m.group(1)), int(m.group(2) or 0)) if m else (-1, -1)
    suffix = pmc_suffix(preset, log2_T, n_rays)  # tools/gpu_pmc.sh PRESET=... LOG2T=...
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*pmc_traffic{suffix}.json")), key=order)
    if not files:
        return None, None, None
    d = json.load(open(files[-1]))
    hits = [v for k, v in d["kernels"].items()
            if any(k.startswith(p) for p in kernel_prefix) and not any(k.startswith(x) for x in GRID_BW_EXCLUDE)]
    if not hits:
        return None, None, None
    req = [v.get("atomic_requests") for v in hits]
    return (round(sum(v["traffic_bytes"] for v in hits)), sum(req) if all(r is not None for r in req) else None,
            os.path.relpath(files[-1], ROOT))


def stage_times(events, steps):
    out = {}
    for ev in events:
        for (a, ea), (b, eb) in zip(ev[:-1], ev[1:]):
            out[b] = out.get(b, 0.0) + ea.elapsed_time(eb)
    return {k: v / steps for k, v in out.items()}


# ---------------------------------------------------------------------------- CPU baseline
def cpu_baseline(n_rays, log2_T, seconds, grid="Hash", n_tables=1, width=64, lr=1e-2, min_timed=2):
    """The reference's hot path restated on the host (oracle/): C march + compositing, fp32 torch
    grid encoding + MLPs with autograd, fused loss, Adam.  Timed on a bounded sample: one untimed
    step, then steps until `seconds` have passed and at least `min_timed` were timed."""
    from mfnerf import synthetic
    from oracle import field_oracle as FO
    from oracle import vren_oracle as O

    # the box's CPU share (OMP_NUM_THREADS is set to it there); os.cpu_count() is the whole host
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
    b = math.exp(math.log(2048 * 0.5 / 16) / 15)
    lay = FO.GridLayout(16, 2, log2_T, 16, b, grid, n_tables)
    g = torch.Generator().manual_seed(0)
    table = torch.empty(lay.n_params).uniform_(-1e-4, 1e-4, generator=g).requires_grad_(True)
    px = FO.xavier_uniform_(torch.empty(3072), FO.mlp_shapes(32, 16, 64, 1), g).requires_grad_(True)
    n_rgb = width * 32 + width * width + 16 * width
    pr = FO.xavier_uniform_(torch.empty(n_rgb), FO.mlp_shapes(32, 3, width, 2), g).requires_grad_(True)
    opt = torch.optim.Adam([px, pr, table], lr=lr, eps=1e-15)
    bf = synthetic.packbits_np(synthetic.ball_density_grid(), 0.01 * 1024 / math.sqrt(3))
    poses = synthetic.camera_poses()
    steps, t0 = 0, None
    while True:
        o, d = synthetic.random_rays(n_rays, poses, seed=steps)
        gt = torch.rand(n_rays, 3, generator=g)
        if steps == 1:
            t0 = time.time()  # first step warms the allocator/threads
        _, ht, _ = O.ray_aabb_intersect(o, d, torch.zeros(1, 3), torch.full((1, 3), 0.5), 1)
        ht[(ht[:, 0, 0] >= 0) & (ht[:, 0, 0] < 0.01), 0, 0] = 0.01
        ra, x, dd, de, ts, cnt = O.raymarching_train(o, d, ht[:, 0].contiguous(), bf, 1, 0.5, 0.0,
                                                     torch.rand(n_rays, generator=g), 128, 1024)
        n = int(cnt[0])
        x, dd, de, ts = x[:n], dd[:n], de[:n].contiguous(), ts[:n].contiguous()
        feat = FO.grid_encode(x + 0.5, table, lay)
        h = FO.mlp_forward(feat, px, 32, 16, 64, 1)
        sigma = torch.exp(h[:, 0])
        dn = dd / dd.norm(dim=1, keepdim=True)
        rgbs = FO.mlp_forward(torch.cat([FO.sh4((dn + 1) / 2), h], 1), pr, 32, 3, width, 2, "ReLU", "Sigmoid")
        s_d, c_d = sigma.detach().contiguous(), rgbs.detach().contiguous()
        tot, op, dep, rgb, ws = O.composite_train_fw(s_d, c_d, de, ts, ra, 1e-4)
        pred = rgb + (1 - op)[:, None]
        e = pred - gt
        dL_drgb = 2 * e / (3 * n_rays)
        o_ = op + 1e-10
        dL_dop = -(dL_drgb.sum(1)) + 1e-3 * (-(torch.log(o_) + 1)) / n_rays
        dsig, drgb = O.composite_train_bw(dL_dop.contiguous(), torch.zeros(n_rays), dL_drgb.contiguous(),
                                          torch.zeros(n), s_d, c_d, ws, de, ts, ra, op, dep, rgb, 1e-4)
        opt.zero_grad()
        torch.autograd.backward([sigma, rgbs], [dsig, drgb])
        opt.step()
        steps += 1
        if t0 is not None and time.time() - t0 >= seconds and steps - 1 >= min_timed:
            break
    el = time.time() - t0
    return {"value": round(n_rays * (steps - 1) / el, 2), "unit": "rays/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{steps - 1} timed training steps x {n_rays} rays, Lego-like synthetic batch, {grid} L16 T2^{log2_T}"
                      f" rgb {width}x2,"
                      f" fp32 torch-CPU field + C oracle march/compositing ({el:.1f} s)"}


def line_base(args, pre, world, elapsed, mean_samples, dp_on=False):
    """The driver-contract fields of the JSON line (value = rays of ALL ranks / slowest rank's time)."""
    rays_total = args.n_rays * args.steps * world
    return {
        "metric": "training rays/sec + test PSNR, Synthetic-NeRF Lego 30k steps" if args.preset == "lego"
                  else "training rays/sec, Synthetic-NeRF MixedFeature rgb-128 (BASELINE config 3 field)",
        "value": round(rays_total / elapsed, 1), "unit": "rays/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f16-mfma/f32",
        "data": "synthetic: 100 analytic 800x800 views of a 12-ball scene (Lego intrinsics), batch drawn on "
                "the device every step; ball-union occupancy (no dataset in the image)",
        "config": {"workload": "%s training step, %d rays/batch/GPU, %s L16 F2 T2^%d%s, rgb %dx2"
                   % ("Lego 800x800" if args.preset == "lego" else "Synthetic-NeRF (MF benchmark field)",
                      args.n_rays, pre["grid"], args.log2_T,
                      " %d tables" % pre["N_tables"] if pre["grid"] == "MixedFeature" else "", pre["rgb_width"]),
                   "preset": args.preset, "global_batch": args.n_rays * world,
                   "rm_s": round(mean_samples / args.n_rays, 2),
                   "parallelism": f"dp{world}" + ("-sharded-adam" if dp_on and args.dp == "shard" else "")
                   + ("-rehearsal" if args.dp_rehearse and world == 1 else ""),
                   "psnr": None},
    }


def resolve_preset(args):
    pre = dict(PRESETS[args.preset])
    if args.n_rays is not None:
        pre["n_rays"] = args.n_rays
    if args.log2_T is not None:
        pre["log2_T"] = args.log2_T
    args.n_rays, args.log2_T = pre["n_rays"], pre["log2_T"]
    return pre


def stub_main(args, world, rank, out_fd):
    """--stub-step: the N-rank plumbing of main() (process group, barrier-bracketed timed region,
    max over ranks, rank 0's single line) around a host-only stand-in step, over gloo, so that the
    launcher is testable without a GPU.  Its line says data "stub"; it is never a measurement."""
    import torch.distributed as dist
    pre = resolve_preset(args)
    if world > 1:
        dist.init_process_group("gloo", world_size=world, rank=rank)
    x = torch.ones(1 << 12)
    for _ in range(args.warmup):
        x.mul_(1.0)
    if world > 1:
        dist.barrier()
    t0 = time.time()
    for _ in range(args.steps):
        x.mul_(1.0)
        if world > 1:
            dist.all_reduce(x)
            x.div_(world)
    if world > 1:
        dist.barrier()
    elapsed = time.time() - t0
    if world > 1:
        t = torch.tensor([elapsed])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    if rank == 0:
        out = line_base(args, pre, world, max(elapsed, 1e-9), 0.0, dp_on=world > 1)
        out["data"] = "stub (launcher test: no GPU step ran)"
        with os.fdopen(out_fd, "w") as f:
            f.write(json.dumps(out) + "\n")
    if world > 1:
        dist.destroy_process_group()


def main(argv=None):
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # N ranks requested without an outer launcher: start one (a child process, no HIP call yet)
        return launch_ranks(args.gpus, sys.argv[1:] if argv is None else argv)
    world = int(env_world or "1")
    if world != args.gpus:
        sys.stderr.write(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: the line would mislabel the run\n")
        return 2
    # the driver reads ONE JSON line from stdout: everything else the process prints there (RCCL's
    # version banner at communicator init, library chatter) goes to stderr; the line itself is
    # written to the original stdout
    out_fd = os.dup(1)
    os.dup2(2, 1)
    sys.stdout = os.fdopen(os.dup(2), "w")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stub_step:
        stub_main(args, world, rank, out_fd)
        return 0
    dp_on = world > 1 or args.dp_rehearse
    if dp_on:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", init_method=None if world > 1 else "tcp://127.0.0.1:29533",
                                             world_size=world, rank=rank)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from mfnerf import dp, engine, synthetic
    if args.dp_rehearse:
        dp.rehearse(True)  # the one-rank group's collectives through RCCL (skipped otherwise)
    # the exchange through a direct RCCL communicator on the step's stream, so the whole data-parallel
    # step (collectives included) replays as one HIP graph (mfnerf/rccl.py).  Default: on for the
    # one-rank rehearsal, off at N > 1 (torch.distributed's collectives between two graphs per step)
    # until a multi-GPU run has pinned the direct path against them; MFNERF_DIRECT_RCCL=1 / 0 forces it
    want_direct = os.environ.get("MFNERF_DIRECT_RCCL", "1" if world == 1 else "0") == "1"
    direct = dp_on and want_direct and dp.use_direct_rccl()

    pre = resolve_preset(args)
    cfg = engine.StepConfig(n_parts=args.parts, **pre)
    step = engine.TrainStep(cfg, device=dev, seed=0)  # identical init on every rank
    if dp_on and args.dp == "shard":
        step.shard_optimizer(rank, world, force=args.dp_rehearse)
    step.set_occupancy(synthetic.ball_density_grid())
    # the training data: 100 analytic 800x800 views (Lego intrinsics, cameras on a radius-1.5
    # sphere) of the very balls the calibrated occupancy grid holds, resident in HBM; every step
    # draws its batch on the device (random image + pixel -> rays + rgb) inside its march graph
    from mfnerf import data
    scene = data.BallScene.matching_grid(seed=0)
    imgs, poses, dirs, K = data.ball_scene_views(scene, 100, synthetic.LEGO_W, synthetic.LEGO_F,
                                                 seed=dp.rank_seed(100, rank), device=dev)
    ds = data.DeviceDataset(imgs, poses, dirs, K=K, img_wh=(synthetic.LEGO_W, synthetic.LEGO_H), device=dev,
                            seed=dp.rank_seed(7, rank))  # rank-distinct rays
    del imgs
    step.attach_dataset(ds)
    batches = [None]

    for i in range(args.warmup):
        run_step(step, batches[i % len(batches)], world, allreduce=dp_on)
    # occupancy refresh cost (amortised every 16 steps in the reference), measured separately
    step.update_density_grid(warmup=False)  # first call allocates the refresh scratch
    torch.cuda.synchronize()
    td = time.time()
    for _ in range(10):
        step.update_density_grid(warmup=False)
    torch.cuda.synchronize()
    density_ms = (time.time() - td) / 10 * 1e3
    step.set_occupancy(synthetic.ball_density_grid())  # keep the calibrated workload for the timed steps

    # per-stage breakdown from an eager pass (an event after every kernel stage)
    n_eager = min(args.steps, 50)
    pass_ev = []
    for i in range(n_eager):
        ev = []
        run_step(step, batches[i % len(batches)], world, ev, allreduce=dp_on)
        pass_ev.append(ev)
    torch.cuda.synchronize()
    eager_stage_ms = stage_times(pass_ev, n_eager)

    # the timed region: the step replayed from HIP graphs (launch overhead off the host); the only
    # per-step host work is the batch copy, three graph launches and two pre-created timing events
    # around the grid_bw graph (the roofline kernel)
    from mfnerf import dp as _dp
    ex = _dp.allreduce_mean_ if dp_on else None
    use_graph = not args.eager
    if use_graph:
        step.capture()
        # the first replays of fresh graphs run slow: settle before timing -- both forms the timed
        # steps replay, the one-graph step and the split step whose scatter the events time.
        # (A 20-step line runs ~5 % slower per step than a 200-step one, and that is the workload, not
        # a start-up cost: the model trains during the bench, and once densities are learned rays
        # terminate earlier in compositing, so fewer samples carry a table gradient -- per-step time
        # falls from 0.519 to 0.474 ms over the first ~500 steps of one process, r6m)
        warm_ev = (torch.cuda.Event(enable_timing=True), [torch.cuda.Event(enable_timing=True)
                                                          for _ in range(step.n_parts)])
        for i in range(24):
            step.replay(exchange=ex, grid_bw_events=warm_ev if i % 4 == 1 else None)
    mk = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    gb_ev = [(mk(), [mk() for _ in range(step.n_parts)]) for _ in range(args.steps)]
    eager_ev = []
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    marched0 = int(step.samples_marched)
    t0 = time.time()
    for i in range(args.steps):
        if use_graph:
            # the next step's batch draw + march overlap this step's grid_bw (the last one draws
            # and marches the batch after the timed steps: extra work inside the timed region)
            timed = i % args.roofline_every == 0
            step.replay(exchange=ex, grid_bw_events=gb_ev[i] if timed else None)
        else:
            ev = []
            run_step(step, batches[i % len(batches)], world, ev, allreduce=dp_on)
            eager_ev.append(ev)
    host_s = time.time() - t0  # the host's issue time for the K steps (GPU-bound when well below elapsed)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.time() - t0
    elapsed = dp.max_over_ranks(elapsed, dev)  # the slowest rank's clock
    if use_graph:
        # the parts' grid_bw scatters run back to back (part q+1's chain overlaps part q's): time
        # from the first one's start to the last one's end
        sampled = gb_ev[::args.roofline_every]
        grid_bw_ms = sum(max(a.elapsed_time(b) for b in ends) for a, ends in sampled) / len(sampled)
    else:
        grid_bw_ms = stage_times(eager_ev, args.steps)["grid_bw"]
    # one batch is marched per timed step (the graphs march the next step's batch)
    mean_samples = (int(step.samples_marched) - marched0) / args.steps
    rays_total = args.n_rays * args.steps * world

    # roofline: grid_bw (the dominant kernel), timed by events around it inside the timed region
    dom = "grid_bw"
    # the newest committed PMC summary of this preset's workload
    traffic, atomic_req, traffic_src = pmc_traffic(GRID_BW_KERNEL, args.preset, args.log2_T, args.n_rays)
    dom_bytes = BYTES_PER_SAMPLE[dom] * mean_samples
    achieved = dom_bytes / (grid_bw_ms * 1e-3) / 1e9
    # the bound the scatter actually meets: memory-side atomic requests per second
    atomic = None
    if atomic_req:
        rate = atomic_req / (grid_bw_ms * 1e-3) / 1e9
        atomic = {"requests_per_launch": round(atomic_req), "requests_per_sample": round(atomic_req / mean_samples, 2),
                  "achieved": round(rate, 2), "peak": ATOMIC_REQ_PEAK_G, "unit": "G requests/s",
                  "frac": round(rate / ATOMIC_REQ_PEAK_G, 4)}
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            # the host path on the bench's own batch (8192 rays x ~60 samples, fw+bw+Adam)
            # and on config 1's 256-ray batch, each a bounded sample on the box's CPU share
            hp = (pre["grid"], pre["N_tables"], pre["rgb_width"], pre["lr"])
            cpu = cpu_baseline(args.n_rays, args.log2_T, args.cpu_seconds, *hp, min_timed=1)
            cpu["other_batches"] = [cpu_baseline(256, args.log2_T, args.cpu_seconds / 2, *hp)]
        out = line_base(args, pre, world, elapsed, mean_samples, dp_on)
        out["config"]["exchange"] = (None if not dp_on else "rccl-direct, one graph per step" if direct
                                     else "torch.distributed between graphs")
        out.update({
            "roofline": {"bound": "hbm", "kernel": dom + " (" + "+".join(GRID_BW_KERNEL) + ")",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "timed_launches": (len(range(0, args.steps, args.roofline_every)) if use_graph
                                            else args.steps),
                         "bytes_per_launch": round(dom_bytes), "bytes_per_sample": BYTES_PER_SAMPLE[dom],
                         "samples_per_launch": round(mean_samples), "atomic": atomic},
            "graph": use_graph, "host_issue_ms_per_step": round(host_s / args.steps * 1e3, 4),
            "grid_bw_ms": round(grid_bw_ms, 4),
            # gated marches that gave up waiting (gate.hip): 0 unless a step stalled GATE_TIMEOUT_US
            "gate_timeouts": step.gate_timeouts() if use_graph else None,
            "eager_stage_ms": {k: round(v, 4) for k, v in eager_stage_ms.items()},
            "density_update_ms": round(density_ms, 3),
            # the reference refreshes occupancy every 16 steps (train.py:62,165): rate with it amortised
            "value_with_occupancy_refresh": round(rays_total / (elapsed + args.steps / 16 * density_ms * 1e-3), 1),
            "cpu_baseline": cpu,
        })
        with os.fdopen(out_fd, "w") as f:
            f.write(json.dumps(out) + "\n")
    if dp_on:
        torch.cuda.synchronize()
        dp.use_direct_rccl(False)  # the direct communicator (ncclCommDestroy) before torch's own
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())

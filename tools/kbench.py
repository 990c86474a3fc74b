"""Per-kernel timing on the bench workload (GPU): each stage of one training step relaunched alone
20 times on the live buffers of a real step; prints median/min microseconds per stage.

    python tools/kbench.py [stage ...]      # default: every stage

Variants of a kernel are compared by running this under different MFNERF_* environment knobs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from mfnerf import engine, synthetic  # noqa: E402
from mfnerf._lib import call, ptr, stream  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    # MFNERF_KBENCH_PRESET=mf128: config 3's field (MixedFeature, 8 tables, T 2^20, rgb 128, 16384 rays)
    preset = os.environ.get("MFNERF_KBENCH_PRESET", "lego")
    kw = {} if preset == "lego" else dict(n_rays=16384, log2_T=20, grid="MixedFeature", N_tables=8, rgb_width=128)
    step = engine.TrainStep(engine.StepConfig(**kw), device=dev)
    step.set_occupancy(synthetic.ball_density_grid())
    b = step.make_batches(2, seed=100)
    for i in range(6):
        bench.run_step(step, b[i % 2], 1)
    torch.cuda.synchronize()
    c, mb, m, t = step.cfg, step.state.march, step.state.march.part[0], step.parts[0]
    cap, Np = step.cap_p, step.Np
    batch = step.last_batch
    n_live = int(m.counter[0])
    zeros_samp = torch.zeros(cap, device=dev)
    planes = torch.empty(c.L, cap, 2, dtype=torch.float16, device=dev)
    rowmajor = torch.empty(cap, 2 * c.L, dtype=torch.float16, device=dev)
    s = stream
    # the fixed-point scatter's per-level scales: the last Adam pass zeroed level_l1 for the next step,
    # so recompute it from this step's dL/dfeat (else every contribution rounds to 0 and no atomic
    # is issued: the timing would miss the scatter itself)
    step._level_l1.zero_()
    call("mfnerf_grid_level_l1", ptr(t.dfeat), cap, ptr(m.counter), c.L, ptr(step._level_l1), s())

    side = torch.cuda.Stream(device=dev)

    def two_queues():
        main = torch.cuda.current_stream()
        ev0, ev1 = torch.cuda.Event(), torch.cuda.Event()
        ev0.record(main)
        side.wait_event(ev0)
        with torch.cuda.stream(side):
            stages["grid_bw_coarse"]()
            ev1.record(side)
        stages["grid_bw_binned"]()
        main.wait_event(ev1)

    stages = {
        "grid_fw": lambda: call("mfnerf_grid_encode_fw", ptr(m.xyzs), cap, ptr(m.counter), step.x_min, step.x_range,
                                step.desc, ptr(step.p16[step.off_table:]), ptr(rowmajor), s()),
        "grid_fw_planar": lambda: call("mfnerf_grid_encode_fw_planar", ptr(m.xyzs), cap, ptr(m.counter), step.x_min,
                                       step.x_range, step.desc, ptr(step.p16[step.off_table:]), ptr(planes), cap, s()),
        "field_fw": lambda: call("mfnerf_field_fw", ptr(t.feat), cap, ptr(m.dirs), cap, ptr(m.counter), ptr(step.packed),
                                 c.rgb_width, 0, ptr(t.sigma), ptr(t.rgb_s), s()),
        "composite_fw": lambda: call("mfnerf_composite_train_fw", ptr(t.sigma), ptr(t.rgb_s), ptr(m.deltas),
                                     ptr(m.ts), ptr(m.rays_a), Np, cap, c.T_threshold, ptr(t.total), ptr(t.opacity),
                                     ptr(t.depth), ptr(t.rgb), ptr(t.ws), s()),
        "loss": lambda: call("mfnerf_nerf_loss", ptr(t.rgb), ptr(t.opacity), ptr(batch.rgb), Np, c.n_rays,
                             c.lambda_opacity, 1.0, 1.0, 1.0, ptr(t.dL_drgb), ptr(t.dL_dop), ptr(step.loss_parts[-64:]), s()),
        "composite_bw": lambda: call("mfnerf_composite_train_bw", ptr(t.dL_dop), ptr(t.zeros_ray), ptr(t.dL_drgb),
                                     ptr(zeros_samp), ptr(t.sigma), ptr(t.rgb_s), ptr(t.ws), ptr(m.deltas),
                                     ptr(m.ts), ptr(m.rays_a), ptr(t.opacity), ptr(t.depth), ptr(t.rgb), Np, cap,
                                     c.T_threshold, ptr(t.dsig), ptr(t.drgb_s), s()),
        "composite": lambda: call("mfnerf_composite_train_fused", ptr(t.sigma), ptr(t.rgb_s), ptr(m.deltas), ptr(m.ts),
                                  ptr(m.rays_a), Np, cap, c.T_threshold, ptr(batch.rgb), c.n_rays, c.lambda_opacity,
                                  1.0, 1.0, 1.0, ptr(t.total), ptr(t.opacity), ptr(t.depth), ptr(t.rgb), ptr(t.ws),
                                  ptr(t.dL_drgb), ptr(t.dL_dop), ptr(t.dsig), ptr(t.drgb_s), ptr(step.loss_parts), s()),
        "field_bw": lambda: call("mfnerf_field_bw", ptr(t.feat), cap, ptr(m.dirs), cap, ptr(m.counter), ptr(step.packed),
                                 c.rgb_width, ptr(t.dsig), ptr(t.drgb_s), step.grad_scale, ptr(t.dfeat),
                                 ptr(t.mlp_grad), ptr(t.mlp_grad[step.off_rgb:]), ptr(t.field_ws), None, None, s()),
        "grid_bw": lambda: step._grid_bw(mb, 0),
        # the binned path's two halves: the coarse levels' atomics, the fine levels' partitions
        "grid_bw_coarse": lambda: call("mfnerf_grid_encode_bw_binned", ptr(m.xyzs), cap, ptr(m.counter), step.x_min,
                                       step.x_range, step.desc, ptr(t.dfeat), ptr(step.grads[step.off_table:]),
                                       ptr(t.grid_ws), step._bin_slots(), ptr(step._level_l1), 1, s()),
        "grid_bw_binned": lambda: call("mfnerf_grid_encode_bw_binned", ptr(m.xyzs), cap, ptr(m.counter), step.x_min,
                                       step.x_range, step.desc, ptr(t.dfeat), ptr(step.grads[step.off_table:]),
                                       ptr(t.grid_ws), step._bin_slots(), ptr(step._level_l1), 2, s()),
        # the coarse levels on a second stream beside the partitioned levels (concurrency probe)
        "grid_bw_2q": lambda: two_queues(),
        "grid_finish": lambda: step._grid_finish(0),
        "check": lambda: call("mfnerf_check_finite", ptr(step.grads), step.grads.numel(), ptr(step.finite_status), s()),
        "adam": lambda: step._adam(step.grads, 0, step.n_alloc, False),
        "adam_fixed": step._finish_update,  # fused convert + Adam + repack (state changes: timing only)
        "grid_bw_fused": lambda: step._grid_bw(mb, 0, fuse_adam=True),  # + the partitioned tables' Adam
        "adam_partial": lambda: step._finish_update(partial=True),
        "pack": step._pack,
        "march": lambda: step._march(batch, mb, lambda _n: None),
        # the occupancy refresh (every 16 steps in train.py:165-168) as the trainer replays it
        "occupancy": lambda: step.update_density_grid(warmup=False),
    }
    names = sys.argv[1:] or list(stages)
    cnt = m.rays_a[:, 2]
    print(f"live samples {n_live} ({n_live / c.n_rays:.1f}/ray); samples/ray max {int(cnt.max())}, "
          f"rays > 64: {int((cnt > 64).sum())}, > 256: {int((cnt > 256).sum())}", flush=True)
    for name in names:
        fn = stages[name]
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        print(f"{name:14s} median {ts[10]:8.1f} us   min {ts[0]:8.1f} us", flush=True)


if __name__ == "__main__":
    main()

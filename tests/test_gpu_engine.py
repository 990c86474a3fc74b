"""The fused training step: eager run() vs the captured, pipelined replay() (next step's march on a
side stream under this step's grid_bw).  Same seed -> same noise stream, so march outputs must be
identical step by step (bit-exact, also against the C oracle) and losses equal up to the float
atomics' summation order."""
import numpy as np
import pytest
import torch

from mfnerf import engine, synthetic
from mfnerf._lib import load

pytestmark = pytest.mark.gpu


def _make(gpu, parts=2, **kw):
    kw = {"n_rays": 1024, "log2_T": 16, **kw}
    st = engine.TrainStep(engine.StepConfig(n_parts=parts, **kw), device=gpu, seed=0)
    st.set_occupancy(synthetic.ball_density_grid())
    return st


def _record(st):
    rays_a, xyzs = st.gather_march()[:2]
    return {"noise": st.state.noise.clone(), "n": xyzs.shape[0], "rays_a": rays_a, "xyzs": xyzs,
            "loss": float(st.loss_sum)}


def _gate_state(st):
    """(signals, waits) of the step's gate: the scatter's signals and the polling kernel's tickets."""
    g = st._gate.tolist()
    return g[0], g[1]


def test_timed_and_fused_tail_replays_match_eager(gpu):
    """bench.py alternates replays whose scatter is its own (event-timed) graph with replays that run
    scatter + convert/Adam + repack as one graph: any mix is bit-identical to eager steps."""
    K = 7
    a, b = _make(gpu, 1), _make(gpu, 1)
    batches = a.make_batches(K + 1, seed=5)
    for k in range(K):
        b.run(batches[k])
    a.run(batches[0])
    torch.cuda.synchronize()
    a.capture()
    assert a.graphs.get("grid_bw_tail") is not None
    mk = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    for k in range(1, K):
        ev = (mk(), [mk()]) if k % 3 == 0 else None
        a.replay(batches[k], next_batch=batches[k + 1] if k + 1 < K else None, grid_bw_events=ev)
        if ev is not None:
            torch.cuda.synchronize()
            assert ev[0].elapsed_time(ev[1][0]) > 0
    torch.cuda.synchronize()
    # steps 1, 2, 4, 5 ran as one graph with a gated march (gate.hip); every signal was waited for
    assert a.graphs.get("step") is not None and _gate_state(a) == (4, 4)
    assert a.adam_step == b.adam_step
    assert torch.equal(a.params, b.params) and torch.equal(a.m, b.m) and torch.equal(a.v, b.v)
    assert torch.equal(a.p16, b.p16) and int(a.step_dev) == int(b.step_dev)


def test_gate_waits_times_out_and_absorbs_unwaited_signals(gpu):
    """gate.hip: a wait with no signal gives up after its timeout; a wait behind several signals
    passes at once and absorbs the ones nobody waited for (the pair is back in step)."""
    from mfnerf._lib import call, ptr, stream
    gate = torch.zeros(2, dtype=torch.int32, device=gpu)
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    call("mfnerf_gate_wait", ptr(gate), 3000, stream())
    t1.record()
    torch.cuda.synchronize()
    assert 2.5 <= t0.elapsed_time(t1) <= 50.0 and gate.tolist() == [0, 1]
    for _ in range(3):
        call("mfnerf_gate_signal", ptr(gate), stream())
    t0.record()
    call("mfnerf_gate_wait", ptr(gate), 100000, stream())
    t1.record()
    torch.cuda.synchronize()
    assert t0.elapsed_time(t1) < 5.0 and gate.tolist() == [3, 3]
    with pytest.raises(RuntimeError):
        call("mfnerf_gate_wait", ptr(gate), -1, stream())


@pytest.mark.parametrize("parts", [1, 2, 4])
def test_pipelined_replay_matches_eager(gpu, oracle, parts):
    K = 6
    a, b = _make(gpu, parts), _make(gpu, parts)
    batches = a.make_batches(K + 1, seed=3)
    # eager reference
    ref = []
    for k in range(K):
        b.run(batches[k])
        torch.cuda.synchronize()
        ref.append(_record(b))
    # pipelined graphs: step 0 eager (lazy init), capture, then replays with the next batch pre-marched
    a.run(batches[0])
    torch.cuda.synchronize()
    got = [_record(a)]
    a.capture()
    for k in range(1, K):
        a.replay(batches[k], next_batch=batches[k + 1] if k + 1 < K else None)
        torch.cuda.synchronize()
        got.append(_record(a))
    for k in range(K):
        r, g = ref[k], got[k]
        assert torch.equal(g["noise"], r["noise"]), f"step {k}: noise stream differs"
        assert g["n"] == r["n"] and torch.equal(g["rays_a"], r["rays_a"]) and torch.equal(g["xyzs"], r["xyzs"])
        assert abs(g["loss"] - r["loss"]) <= 1e-3 * abs(r["loss"]), (k, g["loss"], r["loss"])
    if parts == 1:
        # one part: fixed-point table gradient, fused convert+Adam tail, MLP fold on a second stream --
        # all order-fixed, so the replayed training is bit-identical to the eager one
        assert torch.equal(a.params, b.params) and torch.equal(a.m, b.m) and torch.equal(a.p16, b.p16)
    # the march each replay used is the reference's march of that batch with that noise
    k = K - 1
    o, d = batches[k].rays_o.cpu(), batches[k].rays_d.cpu()
    c, h = torch.zeros(1, 3), torch.full((1, 3), 0.5)
    _, ht, _ = oracle.ray_aabb_intersect(o, d, c, h, 1)  # rays of all parts, one march
    t1 = ht[:, 0, 0]
    t1[(t1 >= 0) & (t1 < 0.01)] = 0.01
    out = oracle.raymarching_train(o, d, ht[:, 0].contiguous(), a.bitfield.cpu(), a.cascades, 0.5, 0.0,
                                   got[k]["noise"].cpu(), a.G, 1024)
    rays_a_o, xyzs_o, n_o = out[0], out[1], int(out[5][0])
    assert n_o == got[k]["n"]
    assert torch.equal(got[k]["rays_a"].cpu(), rays_a_o)
    assert torch.equal(got[k]["xyzs"].cpu(), xyzs_o[:n_o])


@pytest.mark.parametrize("kw", [{}, {"grid": "MixedFeature", "N_tables": 8, "rgb_width": 128}],
                         ids=["hash-rgb64", "mixedfeature-rgb128"])
def test_parts_sum_to_the_whole_batch(gpu, kw):
    """n_parts only changes the schedule: the loss and the gradient of one step (before Adam) are
    the same for 1 part (int32 fixed-point table gradient) and 2 / 4 parts (float atomics), up to
    summation order and the fixed-point resolution -- per parameter block (MLPs, table)."""
    out = []
    for parts in (1, 2, 4):
        st = _make(gpu, parts, **kw)
        batch = st.make_batches(1, seed=9)[0]
        st.run(batch, optimize=False)
        torch.cuda.synchronize()
        out.append((float(st.loss_sum), st.grads.clone(), st.gather_march()[0]))
    blocks = [(0, st.off_rgb), (st.off_rgb, st.off_table), (st.off_table, st.n_params)]
    for loss, g, ra in out[1:]:
        assert torch.equal(ra, out[0][2])
        assert abs(loss - out[0][0]) <= 1e-5 * abs(out[0][0])
        for a, b in blocks:
            ref = out[0][1][a:b]
            assert float(ref.abs().max()) > 0
            assert torch.allclose(g[a:b], ref, rtol=1e-3, atol=1e-4 * float(ref.abs().max())), (a, b)


def test_distortion_loss_in_the_fused_step(gpu, oracle):
    """--distortion_loss_w > 0: the step adds lambda*mean(distortion) to the loss and feeds its
    dL/dws into the compositing backward (losses.py:55-58), per part, checked against the oracle."""
    lam = 1e-2
    st = engine.TrainStep(engine.StepConfig(n_rays=512, log2_T=16, n_parts=2, lambda_distortion=lam), device=gpu)
    st.set_occupancy(synthetic.ball_density_grid())
    ref = engine.TrainStep(engine.StepConfig(n_rays=512, log2_T=16, n_parts=2), device=gpu)
    ref.set_occupancy(synthetic.ball_density_grid())
    batch = st.make_batches(1, seed=4)[0]
    st.run(batch)
    ref.run(batch)
    torch.cuda.synchronize()
    dist_total = 0.0
    cpu = lambda x: x.detach().cpu()  # noqa: E731
    for q, t in enumerate(st.parts):
        m = st.state.march.part[q]
        n = int(st.state.counters[q, 0])
        loss, wsi, wtsi = oracle.distortion_loss_fw(cpu(t.ws[:n]), cpu(m.deltas[:n]), cpu(m.ts[:n]), cpu(m.rays_a))
        dist_total += float(loss.sum())
        g = oracle.distortion_loss_bw(torch.full((st.Np,), lam / 512), wsi, wtsi, cpu(t.ws[:n]), cpu(m.deltas[:n]),
                                      cpu(m.ts[:n]), cpu(m.rays_a))
        assert torch.allclose(cpu(t.dL_dws[:n]), g, rtol=1e-4, atol=1e-9)
    # same params, noise and batch in both steps: the losses differ by exactly the distortion term
    assert abs(float(st.loss_sum) - float(ref.loss_sum) - lam * dist_total / 512) <= 1e-5 * float(st.loss_sum)


@pytest.mark.parametrize("kw", [{}, {"grid": "MixedFeature", "N_tables": 8, "rgb_width": 128}],
                         ids=["hash-rgb64", "mixedfeature-rgb128"])
@pytest.mark.parametrize("skip", [False, True])
def test_fused_convert_adam_matches_finish_then_adam(gpu, kw, skip):
    """mfnerf_adam_step_fixed (the graph-replayed tail of an unsharded step) == the finish call
    (fixed-point -> float, private copies folded) followed by mfnerf_adam_step, bit for bit: params,
    m, v, the fp16 mirror, Adam's step counter, and the zeroed gradient and private copies -- also on a
    step skipped for a non-finite gradient."""
    st = _make(gpu, 1, **kw)
    batches = st.make_batches(2, seed=5)
    st.run(batches[0])  # m, v non-zero
    mb, nomark = st.mbuf[0], (lambda name: None)
    st._use(mb)
    st._march(batches[1], mb, nomark)
    st._chain(batches[1], mb, 0, nomark)
    st._grid_bw(mb, 0)
    if skip:
        st.finite_status[0] = 1
    torch.cuda.synchronize()
    names = ("params", "grads", "m", "v", "p16", "step_dev", "finite_status", "_level_l1")
    # the private copies of the dense levels: the workspace's prefix (the binned scatter keeps its
    # scratch -- bin counts, records -- after them)
    from mfnerf._lib import load
    ws = st.parts[0].grid_ws[:max(16, load().mfnerf_grid_encode_bw_workspace(st.desc)) // 4]
    snap = {k: getattr(st, k).clone() for k in names}
    snap_ws = ws.clone()
    assert int((snap["grads"][st.off_table:] != 0).sum()) > 1000 and int((snap_ws != 0).sum()) > 0
    assert bool((snap["_level_l1"] > 0).all())

    st._grid_finish(0)
    st._update()
    torch.cuda.synchronize()
    ref = {k: getattr(st, k).clone() for k in names}
    for k in names:
        getattr(st, k).copy_(snap[k])
    ws.copy_(snap_ws)
    st._finish_update()
    torch.cuda.synchronize()
    for k in names:
        assert torch.equal(getattr(st, k), ref[k]), k
    assert not bool(ws.any()) and not bool(st.grads.any())
    if skip:
        assert torch.equal(st.params, snap["params"]) and int(st.finite_status[1]) == int(snap["finite_status"][1]) + 1
    else:
        assert not torch.equal(st.params, snap["params"])


@pytest.mark.parametrize("kw", [{}, {"grid": "MixedFeature", "N_tables": 8, "rgb_width": 128}],
                         ids=["hash-rgb64", "mixedfeature-rgb128"])
@pytest.mark.parametrize("skip", [False, True])
@pytest.mark.parametrize("mode", ["partial", "all", "all-overflow"])
def test_partitioned_accumulate_with_fused_adam_matches_unfused(gpu, kw, skip, mode):
    """The replayed tail with the partitioned tables' Adam fused into the accumulate
    (partial: mfnerf_grid_encode_bw_binned_adam + mfnerf_adam_step_fixed_partial; all:
    mfnerf_grid_encode_bw_binned_adam_all, the MLPs' and dense levels' update riding the accumulate's
    launch; all-overflow: the same with record slots sized far below the live count, so the atomic
    fallback and the overflow pass run) == the scatter followed by the one-pass convert + Adam
    (mfnerf_adam_step_fixed), bit for bit: params, m, v, the fp16 mirror, the step counter, the
    zeroed gradient words, copies and level_l1 -- also on a skipped step."""
    if mode == "all-overflow":
        # small tables (few partitions) and a full batch: ~480 records per (partition, unit) slot
        # against slots sized for 256 samples (112 records)
        st = engine.TrainStep(engine.StepConfig(n_rays=8192, log2_T=12, n_parts=1, **kw), device=gpu, seed=0)
        st.set_occupancy(synthetic.ball_density_grid())
        st._bin_slots = lambda: 256
    else:
        st = _make(gpu, 1, **kw)
    assert st._fused_adam_ok()
    batches = st.make_batches(2, seed=5)
    st.run(batches[0])  # m, v non-zero
    mb, nomark = st.mbuf[0], (lambda name: None)
    st._use(mb)
    st._march(batches[1], mb, nomark)
    st._chain(batches[1], mb, 0, nomark)
    if skip:
        st.finite_status[0] = 1
    torch.cuda.synchronize()
    names = ("params", "grads", "m", "v", "p16", "step_dev", "finite_status", "_level_l1")
    snap = {k: getattr(st, k).clone() for k in names}
    ws = st.parts[0].grid_ws
    snap_ws = ws.clone()
    st._grid_bw(mb, 0)
    st._finish_update()
    torch.cuda.synchronize()
    ref = {k: getattr(st, k).clone() for k in names}
    ref_ws = ws.clone()
    for k in names:
        getattr(st, k).copy_(snap[k])
    ws.copy_(snap_ws)
    if mode == "partial":
        st._grid_bw(mb, 0, fuse_adam=True)
        st._finish_update(partial=True)
    else:
        st._grid_bw(mb, 0, fuse_adam="all")
        st._pack()
    torch.cuda.synchronize()
    if mode == "all-overflow":
        ovf = load().mfnerf_grid_encode_bw_binned_flag_offset(st.desc, st._bin_slots()) // 4
        # the overflow path really ran: records past full slots went into the table by atomics
        assert int(ws[ovf].view(torch.int32)) > 0
    for k in names:
        got = getattr(st, k)
        if not torch.equal(got, ref[k]):
            d = (got.float() - ref[k].float()).abs()
            bad = torch.nonzero(d.flatten() > 0).flatten()
            raise AssertionError(f"{k}: {bad.numel()} values differ, first {bad[:8].tolist()}, max {float(d.max())}, "
                                 f"off_table {st.off_table}, first partitioned value "
                                 f"{st.off_table + load().mfnerf_grid_binned_first_value(st.desc)}")
    nc = load().mfnerf_grid_encode_bw_workspace(st.desc) // 4  # the private copies: zeroed by both
    assert not bool(ws[:nc].any()) and not bool(ref_ws[:nc].any()) and not bool(st.grads.any())
    if not skip:
        assert not torch.equal(st.params, snap["params"])


def test_gated_replay_with_distortion_loss_keeps_the_gate_in_step(gpu):
    """--distortion_loss_w > 0 composites in two stages (composite_fw / composite_bw, no fused
    kernel): the step graph must still open the gate once per step, else every gated march would spin
    for GATE_TIMEOUT_US (2 ms) first.  Replays stay bit-identical to eager steps."""
    K = 5
    a, b = _make(gpu, 1, lambda_distortion=1e-3), _make(gpu, 1, lambda_distortion=1e-3)
    batches = a.make_batches(K + 1, seed=9)
    for k in range(K):
        b.run(batches[k])
    a.run(batches[0])
    a.capture()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for k in range(1, K):
        a.replay(batches[k], next_batch=batches[k + 1] if k + 1 < K else None)
    t1.record()
    torch.cuda.synchronize()
    # replays 1..K-2 ran as one gated graph (the last has no next batch); every signal waited for
    assert _gate_state(a) == (K - 2, K - 2)
    assert a.gate_timeouts() == 0  # every gated march started on its signal (gate.hip's gate[3])
    assert t0.elapsed_time(t1) < 4 * (K - 1) * engine.GATE_TIMEOUT_US / 1000  # (loose sanity bound)
    assert torch.equal(a.params, b.params) and torch.equal(a.p16, b.p16)


@pytest.mark.parametrize("kw", [{}, {"binned_grid": False}, {"fixed_point_grid": False}],
                         ids=["fused-tail", "atomic-scatter", "float-scatter"])
def test_gated_replay_opens_the_gate_on_every_tail(gpu, kw):
    """The one-graph step opens the gate once per step whichever scatter and optimizer tail it runs:
    the fused partitioned scatter (the dense-level launch opens it), the fixed-point atomic scatter
    (binned_grid=False) and the float-atomic scatter with the unfused finish + Adam
    (fixed_point_grid=False), each with a signal kernel before it (only the fused tail
    opened it).  Replays match eager steps: bit for bit with the fixed-point gradient, to the float
    atomics' summation order without it."""
    K = 5
    a, b = _make(gpu, 1, **kw), _make(gpu, 1, **kw)
    batches = a.make_batches(K + 1, seed=13)
    for k in range(K):
        b.run(batches[k])
    a.run(batches[0])
    a.capture()
    assert a.graphs.get("step") is not None
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for k in range(1, K):
        a.replay(batches[k], next_batch=batches[k + 1] if k + 1 < K else None)
    t1.record()
    torch.cuda.synchronize()
    assert _gate_state(a) == (K - 2, K - 2)
    assert a.gate_timeouts() == 0  # every gated march started on its signal (gate.hip's gate[3])
    assert t0.elapsed_time(t1) < 4 * (K - 1) * engine.GATE_TIMEOUT_US / 1000  # (loose sanity bound)
    if kw.get("fixed_point_grid", True):
        assert torch.equal(a.params, b.params) and torch.equal(a.p16, b.p16) and torch.equal(a.m, b.m)
    else:  # (a near-zero table gradient's sign, hence its Adam step, can follow the summation order)
        assert torch.isfinite(a.params).all()
        assert float((a.params - b.params).norm() / b.params.norm()) < 1e-2


@pytest.mark.parametrize("log2_T", [20, 21])
def test_large_tables_train_with_or_without_partitions(gpu, log2_T):
    """--T 20 / 21 (opt.py:78): 5120 / 10240 table partitions (past the scatter's 4096 LDS-resident
    running counts) keep the partitioned scatter; eager and replayed steps match bit for bit."""
    a, b = _make(gpu, 1, log2_T=log2_T), _make(gpu, 1, log2_T=log2_T)
    batches = a.make_batches(5, seed=11)
    for k in range(4):
        b.run(batches[k])
    a.run(batches[0])
    a.capture()
    for k in range(1, 4):
        a.replay(batches[k], next_batch=batches[k + 1])
    torch.cuda.synchronize()
    assert torch.isfinite(a.params).all() and a.skipped_steps() == 0
    assert torch.equal(a.params, b.params) and torch.equal(a.p16, b.p16)
    lay = a.layout
    supported = load().mfnerf_grid_encode_bw_binned_workspace(a.desc, a._bin_slots()) >= 0
    assert supported and a._binned()


def test_gate_wait_counts_a_timeout(gpu):
    """A wait whose signal never comes gives up after timeout_us and adds 1 to gate[3]; a wait whose
    signal came first adds nothing (the counter bench.py reports as gate_timeouts)."""
    from mfnerf._lib import call, ptr, stream
    g = torch.zeros(4, dtype=torch.int32, device=gpu)
    call("mfnerf_gate_wait", ptr(g), 50, stream())  # no signal: times out after 50 us
    torch.cuda.synchronize()
    assert g.tolist() == [0, 1, 0, 1]
    call("mfnerf_gate_signal", ptr(g), stream())
    call("mfnerf_gate_signal", ptr(g), stream())
    call("mfnerf_gate_wait", ptr(g), 2000, stream())  # ticket 2, signal 2 present: no wait
    torch.cuda.synchronize()
    assert g.tolist() == [2, 2, 0, 1]

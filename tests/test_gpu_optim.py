"""GPU parity of the optimizer side of the training step against torch: the HIP Adam kernels
(mfnerf_adam_step, mfnerf_adam_step_fixed, the sharded update's slice) vs torch.optim.Adam(eps=1e-15)
and the apex FusedAdam formula (train.py:136), with the CosineAnnealingLR schedule (train.py:140-142)
read from the device and the GradScaler skip; and the dynamic loss scale (PL precision=16,
train.py:287 -> torch.cuda.amp.GradScaler: backoff x0.5 on an overflow, growth x2 after
growth_interval clean steps) driven by the real training step."""
import math

import pytest
import torch

from mfnerf import engine, synthetic
from mfnerf._lib import call, load, ptr, stream
from mfnerf.trainer import HParams, cosine_lr

pytestmark = pytest.mark.gpu

B1, B2, EPS = 0.9, 0.999, 1e-15


def f32(x):
    return float(torch.tensor(x, dtype=torch.float32))


def apex_adam(p, g, m, v, t, lr):
    """apex multi_tensor_adam (ADAM_MODE, decay 0) in float64: m/(1-b1^t), v/(1-b2^t),
    p -= lr * m_hat / (sqrt(v_hat) + eps), with the hyper-parameters as the fp32 values the CUDA
    kernel receives (0.999 as fp32 is 0.999 + 1.3e-8, i.e. 1 - b2 off by 1.3e-5 relative)."""
    b1, b2, eps, lr = f32(B1), f32(B2), f32(EPS), f32(lr)
    m.mul_(b1).add_((1 - b1) * g)
    v.mul_(b2).add_((1 - b2) * g * g)
    p.sub_(lr * ((m / (1 - b1 ** t)) / (torch.sqrt(v / (1 - b2 ** t)) + eps)))


def amp_state(dev, scale=65536.0, interval=2000):
    a = torch.zeros(8, dtype=torch.int32)
    a.view(torch.float32)[2] = scale
    a[4] = interval
    a.view(torch.float32)[5], a.view(torch.float32)[6] = 2.0, 0.5
    return a.to(dev)


def amp_scale(a):
    return float(a.view(torch.float32)[2])


def _check(got, ref64, what, rel=2e-6):
    """fp32 state vs its float64 restatement, relative to the tensor's scale (m, v) -- and for
    params, to the size of the updates, by passing the params' scale as lr-sized steps (below)."""
    err = float((got.double().cpu() - ref64).abs().max() / ref64.abs().max())
    assert err < rel, (what, err)


def _check_params(got, ref64, lr_sum, what, tol):
    """params: each element within 2 fp32 ulps of its value plus tol x the summed step sizes (an
    Adam step moves a parameter by ~lr whatever the gradient's scale)."""
    g = got.double().cpu()
    bound = (ref64.abs() * 2.0 ** -22 + tol * lr_sum)
    err = float(((g - ref64).abs() / bound).max())
    assert err < 1.0, (what, err)


def test_adam_step_matches_torch_adam(gpu):
    """mfnerf_adam_step for 6 steps (one skipped on a non-finite flag) vs the apex formula (float64)
    and torch.optim.Adam(eps=1e-15), with the cosine learning rate held on the device, the device
    step counter, gradient zeroing, the fp16 mirror and the GradScaler bookkeeping."""
    n = 100003  # not a multiple of 4: the tail path too
    g0 = torch.Generator().manual_seed(0)
    p_init = torch.randn(n, generator=g0)
    p, m, v = p_init.clone().to(gpu), torch.zeros(n, device=gpu), torch.zeros(n, device=gpu)
    p16 = torch.empty(n, dtype=torch.float16, device=gpu)
    step_dev = torch.zeros(1, dtype=torch.int32, device=gpu)
    lr_dev = torch.zeros(1, device=gpu)
    amp = amp_state(gpu, interval=3)
    pr, mr, vr = p_init.double(), torch.zeros(n, dtype=torch.float64), torch.zeros(n, dtype=torch.float64)
    tp = p_init.double().clone().requires_grad_(True)
    topt = torch.optim.Adam([tp], lr=1e-2, betas=(B1, B2), eps=EPS)
    hp = HParams(num_epochs=6)
    t, lr_sum = 0, 0.0
    for k in range(6):
        lr = cosine_lr(k, hp)
        lr_dev.fill_(lr)
        grad = torch.randn(n, generator=g0) * 10 ** (k - 3)  # magnitudes 1e-3 .. 1e2
        gd = grad.to(gpu)
        skip = k == 3
        if skip:
            amp[0] = 1  # a producer flagged this step's gradient
        before = (p.clone(), m.clone(), int(step_dev))
        call("mfnerf_adam_step", ptr(p), ptr(gd), ptr(m), ptr(v), ptr(p16), n, 1.0, B1, B2, EPS, 1.0, 0,
             ptr(step_dev), ptr(lr_dev), ptr(amp), 1, stream())
        torch.cuda.synchronize()
        assert int((gd != 0).sum()) == 0  # zeroed for the next step, skipped or not
        assert int(amp[0]) == 0 and int(amp[7]) == 0  # flag cleared, ticket re-armed
        if skip:
            assert torch.equal(p, before[0]) and torch.equal(m, before[1]) and int(step_dev) == before[2]
            assert int(amp[1]) == 1
            continue
        t += 1
        assert int(step_dev) == t
        apex_adam(pr, grad.double(), mr, vr, t, lr)
        for gr_ in topt.param_groups:
            gr_["lr"] = lr
        tp.grad = grad.double().clone()
        topt.step()
        lr_sum += lr
        _check_params(p, pr, lr_sum, "apex params", 1e-5)
        _check(m, mr, "m")
        _check(v, vr, "v")
        # torch's Adam uses the exact betas (apex: their fp32 values): 1e-5 of a step apart
        _check_params(p, tp.detach(), lr_sum, "torch.optim.Adam params", 1e-4)
        assert torch.equal(p16, p.half())


def test_adam_step_fixed_matches_torch_adam(gpu):
    """mfnerf_adam_step_fixed (the replayed step's convert + Adam pass): MLP gradients as floats, the
    table's as int32 fixed-point sums (the dense levels' in the private copies), each converted with
    its table's scale 2^(e-30) (l1 < 2^e) and updated like Adam -- vs the float64 apex formula on the
    converted gradient, for 5 steps with a cosine LR and one skipped step; level_l1 and every gradient
    word are zeroed after each call (by the pass's last workgroup)."""
    st = engine.TrainStep(engine.StepConfig(n_rays=256, log2_T=12), device=gpu)
    lay, desc = st.layout, st.desc
    n, off = st.n_alloc, st.off_table
    # the dense levels' private copies: the workspace's prefix (binned-scatter scratch follows)
    ws = st.parts[0].grid_ws.view(torch.int32)[:max(16, load().mfnerf_grid_encode_bw_workspace(desc)) // 4]
    dense_entries = 0
    for l in range(lay.L):
        if lay.res[l] ** 3 > lay.sizes[l] or lay.offsets[l] != dense_entries:
            break
        dense_entries += lay.sizes[l]
    dense_vals = 2 * dense_entries
    total = lay.n_params
    g0 = torch.Generator().manual_seed(1)
    pr = st.params.double().cpu()
    mr, vr = torch.zeros(n, dtype=torch.float64), torch.zeros(n, dtype=torch.float64)
    hp = HParams(num_epochs=5)
    t, lr_sum = 0, 0.0
    for k in range(5):
        lr = cosine_lr(k, hp)
        st.set_lr(lr)
        l1 = torch.rand(lay.L, generator=g0) * 10.0 ** torch.randint(-8, 2, (lay.L,), generator=g0).float()
        st._level_l1.copy_(l1.to(gpu))
        # the conversion the kernel applies: per table region, scale 2^(30-e), l1 < 2^e
        inv = torch.zeros(total, dtype=torch.float32)
        for l in range(lay.L):
            e = math.frexp(float(l1[l]))[1]
            inv[2 * lay.offsets[l]:2 * (lay.offsets[l] + lay.sizes[l])] = 2.0 ** (e - 30)
        mlp = torch.randn(off, generator=g0) * 1e-3
        q = torch.randint(-(1 << 20), 1 << 20, (total,), generator=g0, dtype=torch.int32)
        copies = torch.randint(-(1 << 16), 1 << 16, (8, dense_vals), generator=g0, dtype=torch.int32)
        tab = q.clone()
        tab[:dense_vals] = copies.sum(0)  # the dense prefix comes only from the copies
        # each copy holds an entry's two features as one packed integer f1 * 2^32 + f0 (64-bit adds)
        c64 = copies.view(8, -1, 2).long()
        packed = (c64[..., 1] << 32) + c64[..., 0]
        g_table = tab.float() * inv
        st.grads.zero_()
        st.grads[:off] = mlp.to(gpu)
        st.grads[off:off + total].view(torch.int32).copy_(q.to(gpu))
        ws[:8 * dense_vals].copy_(packed.reshape(-1).view(torch.int32).to(gpu))
        skip = k == 2
        if skip:
            st.finite_status[0] = 1
        p_before = st.params.clone()
        call("mfnerf_adam_step_fixed", ptr(st.params), ptr(st.grads), ptr(st.m), ptr(st.v), ptr(st.p16), n, off,
             desc, ptr(st.parts[0].grid_ws), ptr(st._level_l1), 1.0, B1, B2, EPS, ptr(st.step_dev), ptr(st.lr_dev),
             ptr(st.finite_status), stream())
        torch.cuda.synchronize()
        assert int((st.grads != 0).sum()) == 0 and int((ws != 0).sum()) == 0
        assert int((st._level_l1 != 0).sum()) == 0  # zeroed for the next step's field_bw
        assert int(st.finite_status[0]) == 0 and int(st.finite_status[7]) == 0
        if skip:
            assert torch.equal(st.params, p_before) and int(st.step_dev) == t
            continue
        t += 1
        assert int(st.step_dev) == t
        grad = torch.zeros(n, dtype=torch.float64)
        grad[:off] = mlp.double()
        grad[off:off + total] = g_table.double()
        apex_adam(pr, grad, mr, vr, t, lr)
        lr_sum += lr
        _check_params(st.params, pr, lr_sum, "params", 1e-5)
        assert torch.equal(st.p16, st.params.half())


def test_sharded_adam_slice_matches_torch_adam(gpu):
    """The ZeRO-1 update's local half (TrainStep._adam on this rank's slice of the flat parameters,
    the fp32 master/m/v held only for the slice): 5 steps vs the apex formula on that slice."""
    st = engine.TrainStep(engine.StepConfig(n_rays=256, log2_T=12), device=gpu)
    world = 2
    st.shard_optimizer(1, world)
    rank, lo, hi = st.shard
    g0 = torch.Generator().manual_seed(2)
    pr = st.params[lo:hi].double().cpu()
    mr, vr = torch.zeros(hi - lo, dtype=torch.float64), torch.zeros(hi - lo, dtype=torch.float64)
    other = st.params[:lo].clone()
    hp = HParams(num_epochs=5)
    lr_sum = 0.0
    for k in range(5):
        lr = cosine_lr(k, hp)
        lr_sum += lr
        st.set_lr(lr)
        grad = torch.randn(hi - lo, generator=g0) * 1e-4
        st.g_shard.copy_(grad.to(gpu))
        st._adam(st.g_shard, lo, hi, False)
        torch.cuda.synchronize()
        apex_adam(pr, grad.double(), mr, vr, k + 1, lr)
        _check_params(st.params[lo:hi], pr, lr_sum, "shard params", 1e-5)
        assert torch.equal(st.p16[lo:hi], st.params[lo:hi].half())
    assert torch.equal(st.params[:lo], other)  # the other rank's slice is not touched here
    assert int(st.step_dev) == 5


def _scale_step(gpu, **kw):
    st = engine.TrainStep(engine.StepConfig(n_rays=256, log2_T=14, **kw), device=gpu)
    st.set_occupancy(synthetic.ball_density_grid())
    return st


def test_dynamic_loss_scale_growth_and_backoff(gpu):
    """GradScaler.update() on the device: the scale starts at 2^16, doubles after growth_interval
    clean steps, halves (and the step is skipped) on an overflow; replayed graphs read the same
    device scale."""
    st = _scale_step(gpu, growth_interval=3)
    good = st.make_batches(8, seed=4)
    assert st.loss_scale() == 65536.0
    for b in good[:3]:
        st.run(b)
    torch.cuda.synchronize()
    assert st.skipped_steps() == 0 and st.loss_scale() == 131072.0 and int(st.finite_status[3]) == 0
    bad = st.make_batches(1, seed=9)[0]
    bad.rgb.fill_(float("nan"))
    p0 = st.params.clone()
    st.run(bad)
    torch.cuda.synchronize()
    assert st.skipped_steps() == 1 and st.loss_scale() == 65536.0 and torch.equal(st.params, p0)
    # graph replays: two clean steps, then the scale grows on the third
    st.capture()
    for b in good[3:6]:
        st.replay(b)
    torch.cuda.synchronize()
    assert st.loss_scale() == 131072.0 and st.skipped_steps() == 1 and int(st.step_dev) == 6


def test_dynamic_loss_scale_recovers_from_persistent_overflow(gpu):
    """with a static scale an overflow that the parameters cause repeats every step and
    training silently freezes.  Here a scale far too large overflows the fp16 backward; every such
    step is skipped and halves the scale until the backward is finite again, and training resumes."""
    st = _scale_step(gpu)
    st.reset_loss_scale(2.0 ** 40)
    batches = st.make_batches(4, seed=5)
    steps0 = int(st.step_dev)
    for i in range(40):
        st.run(batches[i % 4])
    torch.cuda.synchronize()
    skipped = st.skipped_steps()
    assert 10 <= skipped < 40, skipped  # backed off from 2^40 by halving
    assert int(st.step_dev) == steps0 + 40 - skipped  # and then every later step was applied
    assert st.loss_scale() == 2.0 ** (40 - skipped)
    assert torch.isfinite(st.params).all()


def test_static_loss_scale_option(gpu):
    """dynamic_loss_scale=False: the fixed power-of-two scale, no growth."""
    st = _scale_step(gpu, dynamic_loss_scale=False, growth_interval=1)
    for b in st.make_batches(3, seed=6):
        st.run(b)
    torch.cuda.synchronize()
    assert st.loss_scale() == st.grad_scale and st.skipped_steps() == 0 and int(st.step_dev) == 3


def test_level_l1_any_level_count(gpu):
    """mfnerf_grid_level_l1 for level counts that do not divide the 64-lane wave."""
    g = torch.Generator().manual_seed(3)
    for L in (4, 12, 16, 20, 28, 32):
        for n in (1, 777, 40000):
            dy = torch.randn(n, 2 * L, generator=g)
            out = torch.zeros(L, device=gpu)
            call("mfnerf_grid_level_l1", ptr(dy.to(gpu)), n, None, L, ptr(out), stream())
            ref = dy.abs().view(n, L, 2).sum((0, 2))
            assert torch.allclose(out.cpu(), ref, rtol=1e-5), (L, n)

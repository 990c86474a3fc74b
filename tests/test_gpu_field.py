"""GPU parity of the grid encoding and the MFMA field head against the fp32 torch oracle
(oracle/field_oracle.py).  tcnn computes in fp16, so the oracle here rounds every MLP operand to
fp16 exactly where the kernels do and the tolerances are fp16-sized (stated per assert)."""
import math
import os

import numpy as np
import pytest
import torch

from conftest import ROOT
from mfnerf import field as FLD
from mfnerf._lib import call, load, ptr, stream
from mfnerf.grid import GridLayout
from oracle import field_oracle as FO

pytestmark = pytest.mark.gpu

LEGO_B = math.exp(math.log(2048 * 0.5 / 16) / 15)

# The partitioned (binned) scatter carries each weighted contribution of the hashed levels as an
# fp16 value (8-B records: the algorithmic fp16 scatter's own payload; tcnn's gradient is an fp16
# SUM, rounded at every add): each contribution is rounded once to 11 significant bits, so an
# entry's error is within 2^-11 of the sum of its contributions' magnitudes -- the oracle's
# gradient of the same encoding taken with |dL/dy| (the interpolation weights are >= 0).
REC_REL = 2.0 ** -11


def _abs_grad(x, dy, olay):
    """Per table entry: the sum over samples of |contribution| (fp64)."""
    ta = torch.zeros(olay.n_params).requires_grad_(True)
    (FO.grid_encode(x, ta, olay).double() * dy.abs().double()).sum().backward()
    return ta.grad.double()


def _table_unit_bound(x, dy, lay, olay):
    """Per parameter: half the fixed-point unit of its table times the number of contributions it
    receives -- the rounding of a partition summed at its table's own unit (a partition whose slot
    overflowed: every contribution rounded once to 2^(e-30), the table's L1 < 2^e)."""
    cnt = torch.zeros(olay.n_params // 2, dtype=torch.float64)
    l1 = (dy.abs().double().view(dy.shape[0], lay.L, 2).sum(2)).sum(0)  # per level
    for lv in FO._corners(x, olay):
        for idx, _ in lv:
            cnt += torch.bincount(idx, minlength=cnt.numel()).double()
    bound = torch.zeros(olay.n_params // 2, dtype=torch.float64)
    for l in range(lay.L):
        t_l1 = float(sum(l1[k] for k in range(lay.L) if lay.offsets[k] == lay.offsets[l]))
        if t_l1 > 0:
            unit = 2.0 ** (math.frexp(t_l1)[1] - 30)
            a, b = lay.offsets[l], lay.offsets[l] + lay.sizes[l]
            bound[a:b] = 0.5 * unit * cnt[a:b]
    return bound.repeat_interleave(2)


def _assert_binned(got, gref, gabs, atol, rtol=0.0, what=None):
    """|got - ref| <= 2^-11 x (sum of |contributions|) + the fixed-point path's own tolerance."""
    got, gref = got.double(), gref.double()
    excess = (got - gref).abs() - (REC_REL * 1.0001 * gabs + atol + rtol * gref.abs())
    assert float(excess.max()) <= 0, (what, float(excess.max()), int(excess.argmax()))


def test_mfma_f16_lane_maps(gpu):
    g = torch.Generator().manual_seed(0)
    A = torch.randint(-4, 5, (32, 16), generator=g).half()
    B = torch.randint(-4, 5, (16, 32), generator=g).half()
    B[3, 7] = 3  # asymmetric
    D = torch.empty(32, 32, device=gpu)
    Ag, Bg = A.to(gpu), B.to(gpu)
    # the probe kernel lives in a test-support library (tests/support), not in the product C-ABI
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "support", "libmfnerf_probe.so"))
    lib.mfnerf_probe_mfma.argtypes = [ctypes.c_void_p] * 4
    assert lib.mfnerf_probe_mfma(Ag.data_ptr(), Bg.data_ptr(), D.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert torch.equal(D.cpu(), A.float() @ B.float())


def _layouts():
    return [("lego_hash", (16, 2, 19, 16, LEGO_B, "Hash", 1)),
            ("small_T_hash", (8, 2, 10, 4, 8 ** (1 / 7), "Hash", 1)),
            ("mixed_feature", (16, 2, 16, 16, LEGO_B, "MixedFeature", 4)),
            # shared tables of 2^8 entries = ONE partition each: an x-pair's XOR mask reaching past the
            # table must not become a pair record (the same-partition test cannot catch it)
            ("mixed_one_partition_tables", (16, 2, 12, 16, LEGO_B, "MixedFeature", 16)),
            # --T 21 (opt.py:78): 10 x 1024 partitions, past the scatter's LDS-resident running counts
            ("hash_T21", (16, 2, 21, 16, LEGO_B, "Hash", 1))]


@pytest.mark.parametrize("name,args", _layouts())
def test_grid_encode_fw_bw(gpu, name, args):
    lay = GridLayout(*args)
    olay = FO.GridLayout(*args)
    assert lay.n_params == olay.n_params and lay.offsets == olay.offsets
    g = torch.Generator().manual_seed(2)
    N = 6000
    x = torch.rand(N, 3, generator=g)
    x[:8] = torch.tensor([0.0, 1.0]).repeat(12)[:24].view(8, 3)  # faces/corners of the unit cube
    table = ((torch.rand(lay.n_params, generator=g) - 0.5)).half().float()
    ref = FO.grid_encode(x, table, olay)
    desc = lay.desc()
    out = FLD.grid_encode_fw(x.to(gpu), N, table.half().to(gpu), lay, desc)
    # fp32 accumulation of fp16 corners, one fp16 rounding of the output: <= 1 fp16 ulp (|y| < 1)
    assert torch.allclose(out.float().cpu(), ref, atol=1e-3, rtol=0)
    # backward: index_add (oracle autograd) vs fp32 atomics
    dy = torch.randn(N, lay.L * lay.F, generator=g)
    tp = table.clone().requires_grad_(True)
    (FO.grid_encode(x, tp, olay) * dy).sum().backward()
    gref = tp.grad
    xg, dyg = x.to(gpu), dy.to(gpu)
    # with the private-copy workspace (the training path) and without
    for ws in (FLD.grid_bw_workspace(desc, gpu), None):
        gt = torch.zeros(lay.n_params, device=gpu)
        FLD.grid_encode_bw(xg, N, dyg, gt, lay, desc, workspace=ws)
        assert torch.allclose(gt.cpu(), gref, rtol=1e-4, atol=1e-4 * float(gref.abs().max()))
        # accumulates (caller zeroes); the workspace is left zero for the next call
        FLD.grid_encode_bw(xg, N, dyg, gt, lay, desc, workspace=ws)
        assert torch.allclose(gt.cpu(), 2 * gref, rtol=1e-4, atol=2e-4 * float(gref.abs().max()))
        if ws is not None:
            assert int((ws != 0).sum()) == 0
    # fixed-point path (int32 atomics, per-level scale from the L1 norm of dy): same sums to the
    # level resolution, and bit-reproducible (integer atomics are order-independent)
    fx = []
    for ws in (FLD.grid_bw_workspace(desc, gpu), None, FLD.grid_bw_workspace(desc, gpu)):
        gt = torch.zeros(lay.n_params, device=gpu)
        FLD.grid_encode_bw(xg, N, dyg, gt, lay, desc, workspace=ws, fixed_point=True)
        assert torch.allclose(gt.cpu(), gref, rtol=1e-4, atol=1e-4 * float(gref.abs().max()))
        if ws is not None:
            assert int((ws != 0).sum()) == 0
        fx.append(gt)
    assert torch.equal(fx[0], fx[1]) and torch.equal(fx[0], fx[2])
    # partitioned LDS scatter (the training path): same fixed point, bit-reproducible, workspace
    # copies left zero
    bn = []
    gabs = _abs_grad(x, dy, olay)
    for _ in range(2):
        ws = FLD.grid_bw_binned_workspace(desc, N, gpu)
        gt = torch.zeros(lay.n_params, device=gpu)
        FLD.grid_encode_bw(xg, N, dyg, gt, lay, desc, workspace=ws, binned=True)
        _assert_binned(gt.cpu(), gref, gabs, 1e-4 * float(gref.abs().max()), rtol=1e-4)
        nc = load().mfnerf_grid_encode_bw_workspace(desc) // 4
        assert int((ws[:nc] != 0).sum()) == 0
        bn.append(gt)
    assert torch.equal(bn[0], bn[1])
    m = 4099  # not a multiple of the 16-sample chunk: the live count comes from the device
    tp = table.clone().requires_grad_(True)
    (FO.grid_encode(x[:m], tp, olay) * dy[:m]).sum().backward()
    n_dev = torch.tensor([m], dtype=torch.int32, device=gpu)
    for ws in (FLD.grid_bw_workspace(desc, gpu), None):
        for fixed in (False, True):
            gt = torch.zeros(lay.n_params, device=gpu)
            FLD.grid_encode_bw(xg, N, dyg, gt, lay, desc, n_dev=n_dev, workspace=ws, fixed_point=fixed)
            assert torch.allclose(gt.cpu(), tp.grad, rtol=1e-4, atol=1e-4 * float(tp.grad.abs().max()))
    gt = torch.zeros(lay.n_params, device=gpu)
    FLD.grid_encode_bw(xg, N, dyg, gt, lay, desc, n_dev=n_dev, workspace=FLD.grid_bw_binned_workspace(desc, N, gpu),
                       binned=True)
    _assert_binned(gt.cpu(), tp.grad, _abs_grad(x[:m], dy[:m], olay), 1e-4 * float(tp.grad.abs().max()), rtol=1e-4)


@pytest.mark.parametrize("args", [(16, 2, 19, 16, LEGO_B, "Hash", 1), (16, 2, 20, 16, LEGO_B, "MixedFeature", 8)],
                         ids=["lego", "mixedfeature-T20"])
def test_grid_encode_bw_along_rays(gpu, args):
    """Training-shaped input: 64 consecutive samples per ray (long runs of equal coarse corners,
    which the in-wave run merging collapses) with a zero-gradient stretch, at the Lego layout and at
    config 3's MixedFeature layout (8 shared tables of 2^17: the coarse shared levels' single
    records merged per run, round 6)."""
    lay = GridLayout(*args)
    olay = FO.GridLayout(*args)
    g = torch.Generator().manual_seed(5)
    R, S = 700, 64
    o = torch.rand(R, 1, 3, generator=g) * 0.5 + 0.25
    d = torch.nn.functional.normalize(torch.randn(R, 1, 3, generator=g), dim=-1)
    x = (o + d * (torch.arange(S).view(1, S, 1) * (3 ** 0.5 / 1024))).clamp(0, 1).reshape(-1, 3).contiguous()
    N = x.shape[0]
    dy = torch.randn(N, 32, generator=g) * 1e-3
    dy[N // 3: N // 3 + 500] = 0.0  # terminated samples: zero gradient, nothing emitted
    table = torch.zeros(lay.n_params).requires_grad_(True)
    (FO.grid_encode(x, table, olay) * dy).sum().backward()
    gref = table.grad
    desc = lay.desc()
    gabs = _abs_grad(x, dy, olay)
    for fixed, binned in ((False, False), (True, False), (True, True)):
        gt = torch.zeros(lay.n_params, device=gpu)
        ws = FLD.grid_bw_binned_workspace(desc, N, gpu) if binned else FLD.grid_bw_workspace(desc, gpu)
        FLD.grid_encode_bw(x.to(gpu), N, dy.to(gpu), gt, lay, desc, workspace=ws, fixed_point=fixed, binned=binned)
        # the fixed-point quantum is 2^-30 of the level's L1 (~1e-3 of one contribution here); the
        # binned path's dense levels round every sample's contribution once (run sums are integer),
        # ~sqrt(contributions) quanta per entry: 2e-4 of the level's largest entry
        if binned:
            _assert_binned(gt.cpu(), gref, gabs, 2e-4 * float(gref.abs().max()), rtol=1e-4)
        else:
            assert torch.allclose(gt.cpu(), gref, rtol=1e-4, atol=1e-4 * float(gref.abs().max()))
    # the training regime: per-sample gradients ~1e-7 of very different size per level; the
    # fixed-point resolution (2^-30 of each level's L1) stays far below fp32's relative error
    dys = dy * torch.logspace(-9, -5, 32).view(1, 32)
    tp = torch.zeros(lay.n_params).requires_grad_(True)
    (FO.grid_encode(x, tp, olay).double() * dys.double()).sum().backward()
    gref = tp.grad.double()
    gabs = _abs_grad(x, dys, olay)
    for binned in (False, True):
        gt = torch.zeros(lay.n_params, device=gpu)
        ws = FLD.grid_bw_binned_workspace(desc, N, gpu) if binned else FLD.grid_bw_workspace(desc, gpu)
        FLD.grid_encode_bw(x.to(gpu), N, dys.to(gpu), gt, lay, desc, workspace=ws, fixed_point=True, binned=binned)
        got = gt.cpu().double()
        # per table region (a MixedFeature table is shared by several levels)
        for l, (a, b) in enumerate(sorted({(2 * lay.offsets[k], 2 * (lay.offsets[k] + lay.sizes[k])) for k in range(16)})):
            scale = float(gref[a:b].abs().max())
            if scale > 0:
                if binned:
                    _assert_binned(got[a:b], gref[a:b], gabs[a:b], 2e-4 * scale, what=l)
                else:  # (a shared MixedFeature table sums two levels' samples at one table unit: 2e-4)
                    err = float((got[a:b] - gref[a:b]).abs().max()) / scale
                    assert err < (1e-4 if args[5] == "Hash" else 2e-4), (l, err)


@pytest.mark.parametrize("n_rays", [90, 2000], ids=["90rays", "2000rays"])
@pytest.mark.parametrize("name,args", [_layouts()[0], _layouts()[2]])
def test_grid_encode_bw_ragged_rays(gpu, name, args, n_rays):
    """Rays of 1..300 samples packed back to back (a live count that is not a multiple of 16 or
    64): coarse-level runs cross the 16-sample chunks and the 64-sample chunks of the dense-level
    kernel -- vs the fp64 oracle, per level, bit-reproducible.  That kernel sizes a wave's window
    from the live count (one chunk up to 64 x 2048 samples, round 6): 2000 rays (~300 k samples,
    three chunks per window) carry the open runs from chunk to chunk inside a window."""
    lay, olay = GridLayout(*args), FO.GridLayout(*args)
    g = torch.Generator().manual_seed(33)
    lens = torch.randint(1, 301, (n_rays,), generator=g)
    lens[:6] = torch.tensor([1, 15, 16, 17, 63, 65])
    xs = []
    for S in lens.tolist():
        o = torch.rand(1, 3, generator=g) * 0.6 + 0.2
        d = torch.nn.functional.normalize(torch.randn(1, 3, generator=g), dim=-1)
        xs.append(o + d * (torch.arange(S).view(S, 1) * (3 ** 0.5 / 1024)))
    x = torch.cat(xs).clamp(0, 1).contiguous()
    N = x.shape[0]
    dy = torch.randn(N, 2 * lay.L, generator=g) * 1e-3
    dy[N // 2: N // 2 + 77] = 0.0
    tp = torch.zeros(lay.n_params).requires_grad_(True)
    (FO.grid_encode(x, tp, olay).double() * dy.double()).sum().backward()
    gref = tp.grad.double()
    gabs = _abs_grad(x, dy, olay)
    # at ~300 k samples the tables' L1 -- and with it the fixed-point unit -- is ~7x the 90-ray case's:
    # the unit's rounding bound (half a unit per contribution, + 1e-5 of the |contributions| for the
    # fp32 products vs fp64) replaces the atomic path's 1e-4 of the region's largest entry and joins
    # the binned path's 2e-4 (its records' fp16 values and 15-bit x weights)
    ub = _table_unit_bound(x, dy, lay, olay) + 1e-5 * gabs if n_rays > 90 else None
    desc = lay.desc()
    outs = []
    for fixed, binned in ((True, False), (True, True), (True, True)):
        gt = torch.zeros(lay.n_params, device=gpu)
        ws = FLD.grid_bw_binned_workspace(desc, N, gpu) if binned else FLD.grid_bw_workspace(desc, gpu)
        FLD.grid_encode_bw(x.to(gpu), N, dy.to(gpu), gt, lay, desc, workspace=ws, fixed_point=fixed, binned=binned)
        got = gt.cpu().double()
        cuts = sorted(set(2 * o for o in lay.offsets)) + [lay.n_params]  # one region per table
        for a, b in zip(cuts[:-1], cuts[1:]):
            scale = float(gref[a:b].abs().max())
            if scale > 0:  # fixed point: quanta of 2^-30 of the table's L1 (see test_grid_encode_bw_along_rays)
                if binned:
                    _assert_binned(got[a:b], gref[a:b], gabs[a:b], 2e-4 * scale + (0.0 if ub is None else ub[a:b]),
                                   what=(name, a))
                elif ub is None:
                    assert float((got[a:b] - gref[a:b]).abs().max()) <= 1e-4 * scale, (name, a)
                else:
                    excess = (got[a:b] - gref[a:b]).abs() - ub[a:b]
                    assert float(excess.max()) <= 0, (name, a, float(excess.max()))
        outs.append(gt)
    assert torch.equal(outs[1], outs[2])


def test_grid_encode_bw_fixed_point_extreme_range(gpu):
    """No int32 overflow whatever the gradient magnitude (the scale follows the L1 bound), and an
    all-zero gradient leaves the table gradient zero."""
    lay = GridLayout(16, 2, 14, 16, LEGO_B)
    olay = FO.GridLayout(16, 2, 14, 16, LEGO_B)
    g = torch.Generator().manual_seed(9)
    N = 3000
    x = torch.rand(N, 3, generator=g)
    desc = lay.desc()
    for mag in (1e-30, 1e-3, 1e12, 1e30):
        dy = torch.randn(N, 32, generator=g) * mag
        tp = torch.zeros(lay.n_params).requires_grad_(True)
        (FO.grid_encode(x, tp, olay).double() * dy.double()).sum().backward()
        gref = tp.grad.double()
        gabs = _abs_grad(x, dy, olay)
        for binned in (False, True):
            gt = torch.zeros(lay.n_params, device=gpu)
            ws = FLD.grid_bw_binned_workspace(desc, N, gpu) if binned else FLD.grid_bw_workspace(desc, gpu)
            FLD.grid_encode_bw(x.to(gpu), N, dy.to(gpu), gt, lay, desc, workspace=ws, fixed_point=True, binned=binned)
            got = gt.cpu().double()
            assert torch.isfinite(got).all()
            if binned:
                _assert_binned(got, gref, gabs, 1e-4 * float(gref.abs().max()), what=mag)
            else:
                assert float((got - gref).abs().max()) <= 1e-4 * float(gref.abs().max()), mag
    gt = torch.ones(lay.n_params, device=gpu) * 0
    FLD.grid_encode_bw(x.to(gpu), N, torch.zeros(N, 32, device=gpu), gt, lay, desc, fixed_point=True)
    assert int((gt != 0).sum()) == 0


def test_grid_encode_bw_binned_slot_overflow_falls_back(gpu):
    """Pathological input for the partitioned scatter: every sample at one of two points, so each
    level's records pile into a few partitions and overflow their fixed slots; the device then
    scatters the partitioned levels by atomics instead -- same sums (vs the fp64 oracle)."""
    lay = GridLayout(16, 2, 19, 16, LEGO_B)
    olay = FO.GridLayout(16, 2, 19, 16, LEGO_B)
    g = torch.Generator().manual_seed(17)
    N = 40000
    x = torch.tensor([[0.31, 0.42, 0.53], [0.77, 0.12, 0.64]])[torch.randint(0, 2, (N,), generator=g)]
    dy = torch.randn(N, 32, generator=g) * 1e-3
    tp = torch.zeros(lay.n_params).requires_grad_(True)
    (FO.grid_encode(x, tp, olay).double() * dy.double()).sum().backward()
    gref = tp.grad.double()
    desc = lay.desc()
    gt = torch.zeros(lay.n_params, device=gpu)
    FLD.grid_encode_bw(x.to(gpu), N, dy.to(gpu), gt, lay, desc, workspace=FLD.grid_bw_binned_workspace(desc, N, gpu),
                       binned=True)
    _assert_binned(gt.cpu(), gref, _abs_grad(x, dy, olay), 1e-4 * float(gref.abs().max()))


@pytest.mark.parametrize("div", [1, 2, 16])
def test_grid_encode_bw_binned_slots_sized_below_the_count(gpu, div):
    """The record slots sized for n_slots = n / div samples (a training step sizes them for its
    expected count, not its capacity): a live count within ~3x of it still bins; far above it the
    slots overflow and the device falls back to atomics -- the same sums either way."""
    lay = GridLayout(16, 2, 19, 16, LEGO_B)
    olay = FO.GridLayout(16, 2, 19, 16, LEGO_B)
    g = torch.Generator().manual_seed(21)
    N = 20000
    x = torch.rand(N, 3, generator=g)
    dy = torch.randn(N, 32, generator=g) * 1e-3
    tp = torch.zeros(lay.n_params).requires_grad_(True)
    (FO.grid_encode(x, tp, olay).double() * dy.double()).sum().backward()
    gref = tp.grad.double()
    desc = lay.desc()
    ns = N // div
    ws = FLD.grid_bw_binned_workspace(desc, ns, gpu)
    assert ws.numel() * 4 == max(16, load().mfnerf_grid_encode_bw_binned_workspace(desc, ns))
    gt = torch.zeros(lay.n_params, device=gpu)
    FLD.grid_encode_bw(x.to(gpu), N, dy.to(gpu), gt, lay, desc, workspace=ws, binned=True, n_slots=ns)
    _assert_binned(gt.cpu(), gref, _abs_grad(x, dy, olay), 1e-4 * float(gref.abs().max()))


@pytest.mark.parametrize("div", [1, 16])
def test_grid_encode_bw_binned_float_matches_scatter_and_finish(gpu, div):
    """mfnerf_grid_encode_bw_binned_float (the data-parallel step's form: the accumulate writes the
    partitioned tables' floats, one finish pass covers the values before them) gives the same floats,
    bit for bit, as mfnerf_grid_encode_bw_binned + mfnerf_grid_encode_bw_finish -- with the slots
    sized for the count (div 1) and far below it (div 16: records overflow into the workspace's
    words), and with stale values in the partitioned region of the output, which it overwrites."""
    lay = GridLayout(16, 2, 19, 16, LEGO_B)
    g = torch.Generator().manual_seed(23)
    N = 20000
    x = torch.rand(N, 3, generator=g).to(gpu)
    dy = (torch.randn(N, 32, generator=g) * 1e-3).to(gpu)
    desc = lay.desc()
    ns = N // div
    first = load().mfnerf_grid_binned_first_value(desc)
    assert 0 < first < lay.n_params
    ref = torch.zeros(lay.n_params, device=gpu)
    FLD.grid_encode_bw(x, N, dy, ref, lay, desc, workspace=FLD.grid_bw_binned_workspace(desc, ns, gpu), binned=True,
                       n_slots=ns)
    ws = FLD.grid_bw_binned_workspace(desc, ns, gpu)
    out = torch.zeros(lay.n_params, device=gpu)
    for rep in range(2):  # the second call finds the first one's floats in the partitioned region
        if rep:
            out[:first].zero_()
        l1 = torch.zeros(lay.L, device=gpu)
        call("mfnerf_grid_level_l1", ptr(dy), N, None, lay.L, ptr(l1), stream())
        call("mfnerf_grid_encode_bw_binned_float", ptr(x), N, None, 0.0, 1.0, desc, ptr(dy), ptr(out), ptr(ws), ns,
             ptr(l1), None, None, 0, 0, 0, stream())
        torch.cuda.synchronize()
        assert torch.equal(out, ref), f"call {rep}: {int((out != ref).sum())} values differ"
    # the shard flag folded into the finish: a flat gradient [64 MLP values | table] cut into 3
    # shards whose first values fall in the MLP part, the finish's prefix and the partitioned part
    T0 = 64
    flat_n = T0 + lay.n_params
    for raised in (0, 1):
        for shard_len, world in ((T0 + first // 2, 2), (flat_n // 3 // 4 * 4, 3), (T0 + 4, 5)):
            flat = torch.zeros(flat_n, device=gpu)
            flat[:T0] = 1.0
            flag = torch.tensor([raised], dtype=torch.int32, device=gpu)
            l1 = torch.zeros(lay.L, device=gpu)
            call("mfnerf_grid_level_l1", ptr(dy), N, None, lay.L, ptr(l1), stream())
            call("mfnerf_grid_encode_bw_binned_float", ptr(x), N, None, 0.0, 1.0, desc, ptr(dy), ptr(flat[T0:]),
                 ptr(ws), ns, ptr(l1), None, ptr(flag), world, shard_len, T0, stream())
            torch.cuda.synchronize()
            want = torch.cat([torch.ones(T0, device=gpu), ref])
            heads = [k * shard_len for k in range(world) if k * shard_len < flat_n]
            if raised:
                want[heads] = float("nan")
            assert torch.equal(torch.isnan(flat), torch.isnan(want)), (raised, world, shard_len)
            keep = ~torch.isnan(want)
            assert torch.equal(flat[keep], want[keep]), (raised, world, shard_len)


def test_grid_encode_world_coords_normalisation(gpu):
    lay = GridLayout(16, 2, 19, 16, LEGO_B)
    olay = FO.GridLayout(16, 2, 19, 16, LEGO_B)
    g = torch.Generator().manual_seed(3)
    xw = torch.rand(4096, 3, generator=g) - 0.5
    table = ((torch.rand(lay.n_params, generator=g) - 0.5)).half().float()
    xmin, xmax = -torch.ones(1, 3) * 0.5, torch.ones(1, 3) * 0.5
    ref = FO.grid_encode((xw - xmin) / (xmax - xmin), table, olay)  # networks.py:105
    out = FLD.grid_encode_fw(xw.to(gpu), 4096, table.half().to(gpu), lay, lay.desc(), -0.5, 1.0)
    assert torch.allclose(out.float().cpu(), ref, atol=1e-3, rtol=0)


def _field_inputs(N, seed=4, wscale=3.0, width=64):
    g = torch.Generator().manual_seed(seed)
    feat = (torch.rand(N, 32, generator=g) - 0.5).half()
    dirs = torch.randn(N, 3, generator=g)
    px = FO.xavier_uniform_(torch.empty(3072), FO.mlp_shapes(32, 16, 64, 1), g) * wscale
    pr = FO.xavier_uniform_(torch.empty(FLD.rgb_net_params(width)), FO.mlp_shapes(32, 3, width, 2), g) * wscale
    return feat, dirs, px, pr


@pytest.mark.parametrize("N,width", [(1, 64), (31, 64), (33, 64), (5000, 64), (1, 128), (33, 128), (5000, 128)])
def test_field_fw(gpu, N, width):
    # width 128 at 3x Xavier: activations in the hundreds, where an fp16 rounding flip of one hidden
    # unit (accumulation order) moves a logit by ~0.1 -- keep the Xavier scale there
    feat, dirs, px, pr = _field_inputs(N, width=width, wscale=3.0 if width == 64 else 1.0)
    s_ref, c_ref, _ = FO.ngp_field_fw16(feat, dirs, px, pr, width)
    packed = FLD.pack_field_weights(px.to(gpu), pr.to(gpu), width)
    s, c = FLD.field_fw(feat.to(gpu), dirs.to(gpu), N, packed, width)
    # h0 is one fp16 value on both sides; sigma = exp(h0): fp16-accumulation-order noise only
    assert torch.allclose(s.cpu(), s_ref, rtol=4e-3, atol=1e-6)
    assert torch.allclose(c.cpu(), c_ref, atol=2e-3, rtol=0)
    sd, _ = FLD.field_fw(feat.to(gpu), None, N, packed, width, density_only=True)
    assert torch.equal(sd.cpu(), s.cpu())


def test_field_width_unsupported(gpu):
    with pytest.raises(RuntimeError):
        FLD.pack_field_weights(torch.zeros(3072, device=gpu), torch.zeros(FLD.rgb_net_params(96), device=gpu), 96)


def _fp32_autograd(feat, dirs, px, pr, dsig, drgb, width=64):
    f32 = feat.float().requires_grad_(True)
    a = px.half().float().requires_grad_(True)
    b = pr.half().float().requires_grad_(True)
    W = width
    W1 = a[:2048].view(64, 32); W2 = a[2048:3072].view(16, 64)
    R1 = b[:W * 32].view(W, 32); R2 = b[W * 32:W * 32 + W * W].view(W, W); R3 = b[W * 32 + W * W:].view(16, W)
    y1 = torch.relu(f32 @ W1.t()); h = y1 @ W2.t()
    sigma = torch.exp(h[:, 0])
    dn = dirs / torch.norm(dirs, dim=1, keepdim=True)
    r1 = torch.relu(torch.cat([FO.sh4((dn + 1) / 2), h], 1) @ R1.t()); r2 = torch.relu(r1 @ R2.t())
    c = torch.sigmoid(r2 @ R3.t())[:, :3]
    ((sigma * dsig).sum() + (c * drgb).sum()).backward()
    return f32.grad, a.grad, b.grad


@pytest.mark.parametrize("wscale,sig_on,width", [(1.0, 0.0, 64), (1.0, 1.0, 64), (3.0, 1.0, 64), (1.0, 1.0, 128),
                                                 (3.0, 1.0, 128)])
def test_field_bw(gpu, wscale, sig_on, width):
    N = 3000
    feat, dirs, px, pr = _field_inputs(N, seed=5, wscale=wscale, width=width)
    g = torch.Generator().manual_seed(6)
    dsig = torch.randn(N, generator=g) * 1e-6 * sig_on
    drgb = torch.randn(N, 3, generator=g) * 1e-5
    S = 16384.0
    sig, _, acts = FO.ngp_field_fw16(feat, dirs, px, pr, width)
    ref16 = FO.ngp_field_bw16(acts, dsig, drgb, S)
    ref32 = _fp32_autograd(feat, dirs, px, pr, dsig, drgb, width)
    packed = FLD.pack_field_weights(px.to(gpu), pr.to(gpu), width)
    dfeat = torch.empty(N, 32, device=gpu)
    gx = torch.zeros(3072, device=gpu)
    gr = torch.zeros(FLD.rgb_net_params(width), device=gpu)
    ws = FLD.field_bw_workspace(N, width, gpu)
    FLD.field_bw(feat.to(gpu), dirs.to(gpu), N, packed, dsig.to(gpu), drgb.to(gpu), S, dfeat, gx, gr, ws, width)
    for got, r16, r32 in zip((dfeat.cpu(), gx.cpu(), gr.cpu()), ref16, ref32):
        # vs the fp16-point emulation: only fp32 summation-order differences remain
        err = float((got - r16).abs().max() / r16.abs().max())
        assert err < 2e-3, err
        # vs pure fp32 autograd: the fp16 quantisation tcnn's backward has too (~1% rms)
        cos = float(torch.nn.functional.cosine_similarity(got.flatten(), r32.flatten(), dim=0))
        assert cos > 0.9995, cos
    # the deferred fold: adding into zeros and storing over garbage give the undeferred call's bits
    FLD.field_bw(feat.to(gpu), dirs.to(gpu), N, packed, dsig.to(gpu), drgb.to(gpu), S, dfeat, None, None, ws, width)
    st = stream()
    ax, ar = torch.zeros_like(gx), torch.zeros_like(gr)
    call("mfnerf_field_bw_reduce", width, ptr(ws), ptr(ax), ptr(ar), None, st)
    sx, sr = torch.full_like(gx, float("nan")), torch.full_like(gr, 7.0)
    call("mfnerf_field_bw_reduce_store", width, ptr(ws), ptr(sx), ptr(sr), None, st)
    torch.cuda.synchronize()
    assert torch.equal(ax, gx) and torch.equal(ar, gr)
    assert torch.equal(sx, gx) and torch.equal(sr, gr)


@pytest.mark.parametrize("width", [64, 128])
def test_field_bw_truncexp_clamp(gpu, width):
    """TruncExp (custom_functions.py:162-173): sigma = exp(h0) forward, dL/dh0 = g * exp(clamp(h0,
    -15, 15)) backward.  The xyz head's output row 0 is scaled so that h0 spans about +-40: the
    clamped branch is taken on both sides, and the unclamped exp would overflow the fp16 backward at
    this loss scale (exp(40) * g * S >> 65504; clamped, W2^T dh stays below it)."""
    N = 4000
    feat, dirs, px, pr = _field_inputs(N, seed=21, wscale=1.0, width=width)
    px = px.clone()
    px[2048:2048 + 64] *= 60.0  # W2 row 0 -> h0
    g = torch.Generator().manual_seed(22)
    dsig = torch.randn(N, generator=g) * 1e-6
    drgb = torch.randn(N, 3, generator=g) * 1e-3
    S = 8.0
    sig_ref, _, acts = FO.ngp_field_fw16(feat, dirs, px, pr, width)
    h0 = acts["h"][:, 0]
    assert int((h0 > 15).sum()) > N // 10 and int((h0 < -15).sum()) > 40, "clamp branch not exercised"
    ref16 = FO.ngp_field_bw16(acts, dsig, drgb, S)
    packed = FLD.pack_field_weights(px.to(gpu), pr.to(gpu), width)
    s, _ = FLD.field_fw(feat.to(gpu), dirs.to(gpu), N, packed, width)
    assert torch.allclose(s.cpu(), sig_ref, rtol=4e-3, atol=1e-6)  # exp(h0), not clamped, forward
    dfeat = torch.empty(N, 32, device=gpu)
    gx, gr = torch.zeros(3072, device=gpu), torch.zeros(FLD.rgb_net_params(width), device=gpu)
    flag = torch.zeros(2, dtype=torch.int32, device=gpu)
    FLD.field_bw(feat.to(gpu), dirs.to(gpu), N, packed, dsig.to(gpu), drgb.to(gpu), S, dfeat, gx, gr,
                 FLD.field_bw_workspace(N, width, gpu), width, nonfinite=flag)
    torch.cuda.synchronize()
    assert int(flag[0]) == 0 and torch.isfinite(dfeat).all()
    for got, r16 in zip((dfeat.cpu(), gx.cpu(), gr.cpu()), ref16):
        err = float((got - r16).abs().max() / r16.abs().max())
        assert err < 2e-3, err
    # the samples beyond the clamp: their dL/dh0 term is g*exp(+-15) exactly as the oracle's
    big = (h0.abs() > 15)
    err = float((dfeat.cpu()[big] - ref16[0][big]).abs().max() / ref16[0][big].abs().max())
    assert err < 2e-3, err


@pytest.mark.parametrize("name,args", [_layouts()[0], _layouts()[2]])
def test_planar_encode_and_field_match_row_major(gpu, name, args):
    """The training path's level-major encode (XCD-partitioned, paired x-corner loads) equals the
    row-major tcnn-layout encode bit for bit, and the field kernels read either layout to the same
    outputs and data gradients (bit for bit; the weight gradients' in-workgroup sum runs through
    LDS atomics, so their last bits depend on wave order)."""
    lay = GridLayout(*args)
    desc = lay.desc()
    g = torch.Generator().manual_seed(11)
    N, cap = 5003, 5120
    x = torch.rand(N, 3, generator=g)
    x[:8] = torch.tensor([0.0, 1.0]).repeat(12)[:24].view(8, 3)
    table16 = ((torch.rand(lay.n_params, generator=g) - 0.5)).half().to(gpu)
    xg = x.to(gpu)
    row = FLD.grid_encode_fw(xg, N, table16, lay, desc)
    planes = torch.full((lay.L, cap, 2), float("nan"), dtype=torch.float16, device=gpu)
    n_dev = torch.tensor([N], dtype=torch.int32, device=gpu)
    call("mfnerf_grid_encode_fw_planar", ptr(xg), cap, ptr(n_dev), 0.0, 1.0, desc, ptr(table16), ptr(planes), cap,
         torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(planes[:, :N].permute(1, 0, 2).reshape(N, -1), row)
    if lay.L != 16:
        return
    _, dirs, px, pr = _field_inputs(N, seed=12)
    packed = FLD.pack_field_weights(px.to(gpu), pr.to(gpu))
    dg = dirs.to(gpu)
    s1, c1 = FLD.field_fw(row, dg, N, packed)
    s2 = torch.empty(N, device=gpu)
    c2 = torch.empty(N, 3, device=gpu)
    st = torch.cuda.current_stream().cuda_stream
    call("mfnerf_field_fw", ptr(planes), cap, ptr(dg), N, None, ptr(packed), 64, 0, ptr(s2), ptr(c2), st)
    torch.cuda.synchronize()
    assert torch.equal(s1, s2) and torch.equal(c1, c2)
    # the occupancy refresh's form: density only, each sigma also scattered to tmp[cell] (cell -1:
    # skipped), over the device count's first points only
    M = 3 * N
    cell = torch.randperm(M, generator=g)[:N].int()
    cell[::97] = -1
    cg = cell.to(gpu)
    s3 = torch.full((N,), -1.0, device=gpu)
    tmp = torch.zeros(M, device=gpu)
    n_part = torch.tensor([N - 77], dtype=torch.int32, device=gpu)
    call("mfnerf_field_fw_density_scatter", ptr(planes), cap, N, ptr(n_part), ptr(packed), 64, ptr(s3), ptr(cg),
         ptr(tmp), st)
    torch.cuda.synchronize()
    k = N - 77
    assert torch.equal(s3[:k], s1[:k]) and bool((s3[k:] == -1.0).all())
    ref_tmp = torch.zeros(M)
    keep = cell[:k] >= 0
    ref_tmp[cell[:k][keep].long()] = s1[:k].cpu()[keep]
    assert torch.equal(tmp.cpu(), ref_tmp)
    dsig = (torch.randn(N, generator=g) * 1e-6).to(gpu)
    drgb = (torch.randn(N, 3, generator=g) * 1e-5).to(gpu)
    outs = []
    for feat, stride in ((row, 0), (planes, cap)):
        dfeat = torch.empty(N, 32, device=gpu)
        gx, gr = torch.zeros(3072, device=gpu), torch.zeros(7168, device=gpu)
        ws = FLD.field_bw_workspace(N, 64, gpu)
        call("mfnerf_field_bw", ptr(feat), stride, ptr(dg), N, None, ptr(packed), 64, ptr(dsig), ptr(drgb), 4096.0,
             ptr(dfeat), ptr(gx), ptr(gr), ptr(ws), None, None, st)
        torch.cuda.synchronize()
        outs.append((dfeat, gx, gr))
    assert torch.equal(outs[0][0], outs[1][0])
    for a, b in zip(outs[0][1:], outs[1][1:]):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6 * float(b.abs().max()))


def test_grid_encode_bw_fixed_point_shared_tables(gpu):
    """MixedFeature levels share tables: with per-level gradient magnitudes six decades apart, every
    level adding into a shared table must use that table's scale (the sum of its levels' L1 bounds),
    and the conversion back must use it too -- checked per table region against the oracle."""
    args = _layouts()[2][1]
    lay, olay = GridLayout(*args), FO.GridLayout(*args)
    g = torch.Generator().manual_seed(13)
    N = 4000
    x = torch.rand(N, 3, generator=g)
    dy = torch.randn(N, 32, generator=g) * torch.logspace(-9, -3, 16).repeat_interleave(2).view(1, 32)
    tp = torch.zeros(lay.n_params).requires_grad_(True)
    (FO.grid_encode(x, tp, olay).double() * dy.double()).sum().backward()
    gref = tp.grad.double()
    gabs = _abs_grad(x, dy, olay)
    desc = lay.desc()
    for binned in (False, True):
        gt = torch.zeros(lay.n_params, device=gpu)
        ws = FLD.grid_bw_binned_workspace(desc, N, gpu) if binned else FLD.grid_bw_workspace(desc, gpu)
        FLD.grid_encode_bw(x.to(gpu), N, dy.to(gpu), gt, lay, desc, workspace=ws, fixed_point=True, binned=binned)
        got = gt.cpu().double()
        regions = sorted(set((lay.offsets[l], lay.sizes[l]) for l in range(lay.L)))
        assert len(regions) < lay.L  # some tables are shared
        for off, size in regions:
            a, b = 2 * off, 2 * (off + size)
            scale = float(gref[a:b].abs().max())
            if scale > 0 and binned:
                _assert_binned(got[a:b], gref[a:b], gabs[a:b], 1e-4 * scale, what=off)
            elif scale > 0:
                err = float((got[a:b] - gref[a:b]).abs().max()) / scale
                assert err < 1e-4, (off, err)


@pytest.mark.parametrize("name,args", [_layouts()[0], _layouts()[2], _layouts()[3]])
def test_partitioned_scatter_on_rays_with_overflowing_slots(gpu, name, args):
    """The partitioned scatter on training-shaped rays (Lego layout, MixedFeature's shared tables,
    --T 21's 10 x 1024 partitions) with its record slots sized for the count and 16x below it (most
    partitions overflow: their records go through the overflow words and the partition sums at its
    table's unit): within the record bound of the fp64 oracle plus that unit's rounding, and
    bit-reproducible."""
    lay, olay = GridLayout(*args), FO.GridLayout(*args)
    g = torch.Generator().manual_seed(41)
    R, S = 900, 80
    o = torch.rand(R, 1, 3, generator=g) * 0.6 + 0.2
    d = torch.nn.functional.normalize(torch.randn(R, 1, 3, generator=g), dim=-1)
    x = (o + d * (torch.arange(S).view(1, S, 1) * (3 ** 0.5 / 1024))).clamp(0, 1).reshape(-1, 3).contiguous()
    N = x.shape[0]
    dy = torch.randn(N, 2 * lay.L, generator=g) * 1e-3
    tp = torch.zeros(lay.n_params).requires_grad_(True)
    (FO.grid_encode(x, tp, olay).double() * dy.double()).sum().backward()
    gref = tp.grad.double()
    gabs = _abs_grad(x, dy, olay)
    desc = lay.desc()
    for ns in (N, N // 16):
        out = []
        for _ in range(2):
            gt = torch.zeros(lay.n_params, device=gpu)
            FLD.grid_encode_bw(x.to(gpu), N, dy.to(gpu), gt, lay, desc, workspace=FLD.grid_bw_binned_workspace(desc, ns, gpu),
                               binned=True, n_slots=ns)
            out.append(gt.cpu())
        assert float(out[0].abs().max()) > 0
        assert torch.equal(out[0], out[1]), (name, ns, int((out[0] != out[1]).sum()))
        got = out[1].double()
        # slots 16x too small: most partitions overflow and sum at their table's unit (the shared
        # MixedFeature tables' unit follows the L1 of every level sharing them)
        unit = _table_unit_bound(x, dy, lay, olay) if ns < N else torch.zeros(lay.n_params, dtype=torch.float64)
        cuts = sorted(set(2 * o for o in lay.offsets)) + [lay.n_params]  # one region per table
        for a, b in zip(cuts[:-1], cuts[1:]):
            scale = float(gref[a:b].abs().max())
            if scale > 0:
                _assert_binned(got[a:b], gref[a:b], gabs[a:b], 2e-4 * scale + unit[a:b] * 1.0001, what=(name, ns, a))

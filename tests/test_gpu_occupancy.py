"""GPU checks of the device-only occupancy refresh (mfnerf_occupancy_*) against the CPU
restatement of networks.py:157-271 (oracle/occupancy_oracle.py).

Draws are random (counter hash, not torch's streams), so the cell step is checked by property:
warm-up visits every cell once, uniform draws are valid cells, occupied draws only hit cells above
the threshold and cover them uniformly, and every point sits within half a cell of its cell's
centre.  The update step (scatter, decay/max, mean threshold, packbits) is compared exactly.
"""
import math

import numpy as np
import pytest
import torch

from mfnerf._lib import call, load, ptr, stream
from oracle import occupancy_oracle as OO

pytestmark = pytest.mark.gpu

THR = 0.01 * 1024 / math.sqrt(3)


def _cells(gpu, grid, C, G, scale, M, warmup, seed=0, call_index=0, thr=THR):
    lib = load()
    n = lib.mfnerf_occupancy_points(C, G, M, int(warmup))
    ws = torch.empty(lib.mfnerf_occupancy_workspace(C, G), dtype=torch.uint8, device=gpu)
    xyz = torch.empty(n, 3, device=gpu)
    cell = torch.empty(n, dtype=torch.int32, device=gpu)
    call("mfnerf_occupancy_cells", ptr(grid), C, G, scale, M, int(warmup), thr, seed, call_index, ptr(xyz), ptr(cell),
         ptr(ws), stream())
    torch.cuda.synchronize()
    return xyz.cpu(), cell.cpu(), ws


def _update(gpu, grid, sig, cell, C, G, decay=0.95, count_grid=None, ws=None):
    lib = load()
    g = grid.clone().to(gpu)
    bf = torch.zeros(C * G ** 3 // 8, dtype=torch.uint8, device=gpu)
    tmp = torch.empty(C * G ** 3, device=gpu)
    if ws is None:
        ws = torch.empty(lib.mfnerf_occupancy_workspace(C, G), dtype=torch.uint8, device=gpu)
    cg = count_grid.to(gpu) if count_grid is not None else None
    sig, cell = sig.to(gpu), cell.to(gpu)  # keep the device copies alive until the kernels ran
    call("mfnerf_occupancy_update", ptr(g), ptr(sig), ptr(cell), cell.numel(), C, G, decay,
         ptr(cg) if cg is not None else None, THR, ptr(tmp), ptr(bf), ptr(ws), stream())
    torch.cuda.synchronize()
    return g.cpu(), bf.cpu()


@pytest.mark.parametrize("C,G,scale", [(1, 128, 0.5), (3, 32, 4.0)])
def test_warmup_visits_every_cell_once(gpu, C, G, scale):
    grid = torch.zeros(C, G ** 3, device=gpu)
    xyz, cell, _ = _cells(gpu, grid, C, G, scale, G ** 3 // 4, True)
    assert cell.numel() == C * G ** 3
    assert torch.equal(torch.sort(cell.long()).values, torch.arange(C * G ** 3))
    assert OO.cell_points_ok(xyz, cell, C, G, scale)
    # jitter actually spreads points over the cell (not all at the centre)
    ctr, half = OO.cell_centers(cell, C, G, scale)
    assert ((xyz - ctr).abs() / half[:, None]).mean() > 0.4


@pytest.mark.parametrize("C,G,scale", [(1, 128, 0.5), (2, 32, 1.0)])
def test_uniform_and_occupied_draws(gpu, C, G, scale):
    g = torch.Generator().manual_seed(0)
    grid = torch.rand(C, G ** 3, generator=g) * 2 * THR - THR / 2  # mix of negative, sub- and super-threshold
    occ = grid > THR
    M = G ** 3 // 4
    xyz, cell, _ = _cells(gpu, grid.to(gpu), C, G, scale, M, False, seed=7)
    assert cell.numel() == C * 2 * M
    assert OO.cell_points_ok(xyz, cell, C, G, scale)
    cell = cell.long().reshape(C, 2 * M)
    for c in range(C):
        uni, oc = cell[c, :M], cell[c, M:]
        assert ((uni // G ** 3) == c).all() and ((oc // G ** 3) == c).all()
        # uniform draws hit occupied cells at the occupied fraction (binomial, 6 sigma)
        p = occ[c].float().mean().item()
        hit = occ.reshape(-1)[uni].float().mean().item()
        assert abs(hit - p) < 6 * math.sqrt(p * (1 - p) / M)
        # occupied draws only hit occupied cells, spread uniformly over them
        assert occ.reshape(-1)[oc].all()
        counts = torch.bincount(oc - c * G ** 3, minlength=G ** 3)[occ[c]].double()
        lam = M / occ[c].sum().item()
        assert abs(counts.mean().item() - lam) < 1e-9
        assert abs(counts.var().item() / lam - 1) < 0.1  # Poisson dispersion
    # different call_index -> different draws; same -> identical
    _, cell2, _ = _cells(gpu, grid.to(gpu), C, G, scale, M, False, seed=7, call_index=1)
    _, cell3, _ = _cells(gpu, grid.to(gpu), C, G, scale, M, False, seed=7)
    assert not torch.equal(cell2.long().reshape(C, -1), cell)
    assert torch.equal(cell3.long().reshape(C, -1), cell)


def test_occupied_list_order_and_empty_set(gpu):
    C, G = 2, 32
    grid = torch.zeros(C, G ** 3)
    hot = torch.tensor([5, 77, 4096, G ** 3 - 1])
    grid[0, hot] = 10.0  # cascade 1 empty
    xyz, cell, ws = _cells(gpu, grid.to(gpu), C, G, 1.0, 1000, False)
    cell = cell.long().reshape(C, -1)
    assert set(cell[0, 1000:].tolist()) == set(hot.tolist())
    assert (cell[1, 1000:] == -1).all()  # no occupied cells: nothing drawn (the reference's empty nonzero)
    # the compacted list (workspace) is in ascending morton order, like torch.nonzero
    nblk = (G ** 3 + 4095) // 4096
    off = ((4 * C * nblk + 255) // 256) * 256 + 256
    lst = ws[off:off + 4 * G ** 3].cpu().view(torch.int32)[:4]
    assert lst.tolist() == hot.tolist()


@pytest.mark.parametrize("erode", [False, True])
def test_update_matches_reference(gpu, erode):
    C, G = 2, 64
    g = torch.Generator().manual_seed(3)
    grid = torch.rand(C, G ** 3, generator=g) * 1.2 * THR
    grid[:, ::7] = -1.0  # invisible cells (mark_invisible_cells) are never updated
    n = 40000
    cell = torch.randperm(C * G ** 3, generator=g)[:n].int()  # distinct cells: no write order ambiguity
    cell[::50] = -1
    sig = torch.rand(n, generator=g) * 1.5 * THR
    count_grid = torch.randint(0, 4, (C, G ** 3), generator=g).float() if erode else None
    got_g, got_bf = _update(gpu, grid, sig, cell, C, G, count_grid=count_grid)
    ref_g, thr, ref_bf = OO.update(grid, sig, cell, count_grid=count_grid)
    if erode:  # powf vs torch pow: 1 ulp
        torch.testing.assert_close(got_g, ref_g, rtol=2e-7, atol=0)
    else:
        assert torch.equal(got_g, ref_g)
    # packbits against the reference threshold, ignoring cells within 1e-5 of it (mean summation order)
    near = ((ref_g - thr).abs() <= 1e-5 * abs(thr)).reshape(-1)
    bits = lambda b: torch.from_numpy(np.unpackbits(b.numpy(), bitorder="little").astype(bool))
    assert torch.equal(bits(got_bf)[~near], bits(ref_bf)[~near])
    assert thr < THR  # the mean (not the fixed threshold) was the binding one here


def test_update_no_positive_cell_clears_bitfield(gpu):
    C, G = 1, 32
    grid = -torch.ones(C, G ** 3)
    grid[0, :100] = 0.0
    cell = torch.arange(10, dtype=torch.int32)
    sig = torch.zeros(10)
    got_g, got_bf = _update(gpu, grid, sig, cell, C, G)
    ref_g, thr, ref_bf = OO.update(grid, sig, cell)
    assert math.isnan(thr)
    assert torch.equal(got_g, ref_g) and int(got_bf.sum()) == 0 and torch.equal(got_bf, ref_bf)


def test_engine_refresh_end_to_end(gpu):
    """TrainStep.update_density_grid: warm-up then steady-state refreshes reproduce the restated
    update exactly from the points the device probed (one per distinct drawn cell, sigma from the
    same fused field kernels) -- no duplicate cells, so no write-order ambiguity anywhere."""
    from mfnerf import engine, synthetic
    st = engine.TrainStep(engine.StepConfig(n_rays=512, log2_T=16), device=gpu, seed=0)
    st.set_occupancy(synthetic.ball_density_grid())
    for i, warm in enumerate((True, False, False, False)):
        before = st.density_grid.clone().cpu()
        st.update_density_grid(warmup=warm)
        torch.cuda.synchronize()
        o = st._occ
        n = int(o.count)
        # the draws' device call index advanced once per refresh (by a kernel of its own after the
        # warm-up draws, by the marked-cell compaction after the steady-state ones)
        assert int(o.calls) == i + 1
        # the update's scratch is handed back zero (the refresh runs no fill launch for it)
        assert int(torch.count_nonzero(o.tmp)) == 0
        cap = load().mfnerf_occupancy_points_unique(st.cascades, st.G, st.G ** 3 // 4, int(warm))
        assert 0 < n <= cap
        cell = o.cell[:n].cpu().long()
        # distinct, in morton order (warm-up: every cell) or the unique draw's row-major order
        assert torch.equal(cell, torch.sort(cell).values if warm else _row_major(cell, st.G))
        srt = torch.sort(cell).values
        assert (srt[1:] > srt[:-1]).all()
        if warm:
            assert n == st.cascades * st.G ** 3
        ref_g, thr, ref_bf = OO.update(before, o.sigma[:n].cpu(), cell.int())
        got = st.density_grid.cpu()
        if not torch.equal(got, ref_g):
            # evidence for an intermittent in-suite mismatch (never seen in a fresh process): which
            # cells, what the update's scratch held there, whether they were probed
            bad = torch.nonzero((got != ref_g).flatten()).flatten()[:8]
            tmp = o.tmp.cpu().flatten()
            probed = {int(k): i for i, k in enumerate(cell.tolist())} if bad.numel() else {}
            info = [(int(b), float(got.flatten()[b]), float(ref_g.flatten()[b]), float(before.flatten()[b]),
                     float(tmp[b]), probed.get(int(b)), float(o.sigma[probed[int(b)]]) if int(b) in probed else None)
                    for b in bad]
            raise AssertionError(f"warm={warm} n={n}: {int((got != ref_g).sum())} cells differ; "
                                 f"(cell, got, ref, before, tmp, list index, sigma): {info}")
        assert torch.equal(st.bitfield.cpu().flatten(), ref_bf.flatten())  # thr + packbits in one launch
        assert OO.cell_points_ok(o.xyz[:n].cpu(), cell, st.cascades, st.G, st.cfg.scale)


def _cells_unique(gpu, grid, C, G, scale, M, warmup, ws, seed=0, call_index=0, thr=THR):
    lib = load()
    n = lib.mfnerf_occupancy_points_unique(C, G, M, int(warmup))
    xyz = torch.empty(n, 3, device=gpu)
    cell = torch.empty(n, dtype=torch.int32, device=gpu)
    cnt = torch.zeros(1, dtype=torch.int32, device=gpu)
    call("mfnerf_occupancy_cells_unique", ptr(grid), C, G, scale, M, int(warmup), thr, seed, call_index, ptr(xyz),
         ptr(cell), ptr(cnt), ptr(ws), stream())
    torch.cuda.synchronize()
    k = int(cnt)
    return xyz[:k].cpu(), cell[:k].cpu()


def _row_major(cells, G):
    """cells (cascade * G^3 + morton) in the unique draw's order: ascending row-major cell index
    (x fastest) within each cascade."""
    from oracle import vren_oracle
    c, m = cells // G ** 3, cells % G ** 3
    q = vren_oracle.morton3D_invert(m.cpu().int()).long().to(cells.device)
    key = c * G ** 3 + q[:, 0] + G * (q[:, 1] + G * q[:, 2])
    return cells[torch.argsort(key)]


@pytest.mark.parametrize("C,G,scale", [(1, 128, 0.5), (2, 32, 1.0)])
def test_unique_draw_probes_each_drawn_cell_once(gpu, C, G, scale):
    """mfnerf_occupancy_cells_unique: exactly the distinct cells the plain draw (same seed, call index)
    draws, in ascending row-major order within a cascade, one point each inside its cell with the
    jitter spread over the cell; the byte map is left zero (a repeat gives the same result); an empty
    occupied set adds no cell; the warm-up lists every cell in morton order."""
    g = torch.Generator().manual_seed(5)
    grid = (torch.rand(C, G ** 3, generator=g) * 2 * THR - THR / 2).to(gpu)
    M = G ** 3 // 4
    _, plain, _ = _cells(gpu, grid, C, G, scale, M, False, seed=3, call_index=2)
    ws = torch.zeros(load().mfnerf_occupancy_workspace(C, G), dtype=torch.uint8, device=gpu)
    xyz, cell = _cells_unique(gpu, grid, C, G, scale, M, False, ws, seed=3, call_index=2)
    want = _row_major(torch.unique(plain[plain >= 0].long()), G)
    assert torch.equal(cell.long(), want)
    assert cell.numel() < plain.numel()  # the duplicates are gone
    assert OO.cell_points_ok(xyz, cell, C, G, scale)
    ctr, half = OO.cell_centers(cell, C, G, scale)
    assert ((xyz - ctr).abs() / half[:, None]).mean() > 0.4
    xyz2, cell2 = _cells_unique(gpu, grid, C, G, scale, M, False, ws, seed=3, call_index=2)
    assert torch.equal(cell2, cell) and torch.equal(xyz2, xyz)
    # an empty occupied set: only the uniform draws' cells
    _, plain0, _ = _cells(gpu, torch.zeros_like(grid), C, G, scale, M, False, seed=3, call_index=2)
    _, cell0 = _cells_unique(gpu, torch.zeros_like(grid), C, G, scale, M, False, ws, seed=3, call_index=2)
    assert torch.equal(cell0.long(), _row_major(torch.unique(plain0[plain0 >= 0].long()), G))
    # warm-up: every cell, in (morton) order
    _, cw = _cells_unique(gpu, grid, C, G, scale, M, True, ws)
    assert torch.equal(cw.long(), torch.arange(C * G ** 3))


def test_consecutive_refreshes_draw_independent_cells(gpu):
    """The uniform cells of refresh calls 0, 1, 2 overlap only at the random-coincidence rate."""
    C, G = 1, 128
    grid = torch.zeros(C, G ** 3, device=gpu)
    M = 20000
    cells = []
    for k in range(3):
        _, cell, _ = _cells(gpu, grid, C, G, 0.5, M, False, seed=1, call_index=k)
        cells.append(set(cell[:M].tolist()))
    expect = M * M / G ** 3  # ~190 coincidences between two independent draws
    for a in range(3):
        for b in range(a + 1, 3):
            assert len(cells[a] & cells[b]) < 2 * expect + 50

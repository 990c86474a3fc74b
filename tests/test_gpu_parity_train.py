"""End-to-end training parity with the reference (north_star: "PSNR within 0.2 dB of reference").
The Lego images are not in this image, so the comparison runs the protocol of
tests/parity_protocol.py: BASELINE config 1's shape (64x64 views of the analytic ball scene, 256
rays per batch, Lego's default field), train.py's per-epoch cosine schedule over 10 short epochs,
16 held-out views, the same initial weights, ray batches and march perturbations on both sides.  tests/golden/parity_train.json holds the REFERENCE side: its own
render / NeRFLoss / NGP driven in fp32 on the CPU with the oracle kernels
(tests/golden/make_parity_train.py).  Here this repo's fused MI355X step (fp16 MFMA field, dynamic
loss scale, fixed-point table gradient, HIP Adam) trains from the same start, and the held-out
test-time PSNR (mfnerf.rendering.render(test_time=True), the reference's progressive loop) must
land within 0.2 dB of the reference's."""
import json
import math
import os

import pytest
import torch

import parity_protocol as PP
from conftest import ROOT
from mfnerf import engine
from mfnerf.networks import NGP
from mfnerf.rendering import render

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(ROOT, "tests", "golden", "parity_train.json")
# the loss curves: the two sides' logged batch losses (the same batches) pooled over the seeds and
# over each epoch of the schedule; every epoch's pooled ratio ours / reference within 1 +- this.
# (Single logged losses are not compared once the two trajectories part -- fp16 field vs fp32,
# from step ~100 -- one 256-ray batch's loss then differs by ~30 % between equally good models.)
# What 8 seeds resolve: the per-seed epoch ratios spread with sd 0.13-0.25 (r04: standard error of
# the 8-seed pooled ratio 0.05-0.09 per epoch), so a tighter per-epoch bound would fail on noise;
# the whole run's seed-mean log ratio (below) is the sharper test of a systematic shift.
LOSS_TOL_EPOCH = 0.10
# after the early window: mean over seeds of each seed's mean log(ours / reference) per step within
# +-WHOLE_LOG_TOL and within WHOLE_SE_K standard errors of zero (r04: +0.003, se 0.056)
WHOLE_LOG_TOL, WHOLE_SE_K = 0.10, 2.5
# the early window (steps <= 100, before the trajectories part): the pooled ratio within 1 +- this.
# Both sides start from the same weights on the same batches, so the early losses differ only by the
# fp16 field (~1e-3 relative per value) and the 2^-11 rounding of the table-gradient records
# compounding over the first steps; a systematic gradient error of a few percent shows here first.
EARLY_STEPS, LOSS_TOL_EARLY = 100, 0.02
# the first steps, where the two sides train the same model up to fp16 rounding: EVERY step's loss
# within 1 +- this of the reference's (a gradient error of a few percent shows within a few steps).
# r05 (profiles/r05_parity_train.json, early_deviation_per_step): through step 70 every step of every
# seed is within 0.27 % (0.13 % through step 20); from step ~75 the trajectories part, a few seeds at
# a time (seed 0 at 75, seeds 3/4/7 after 80), as two chaotic runs do -- the 25 % single step (seed
# 3, step 84, its neighbours +0.6 % / -0.8 %) is one of 256 rays predicted differently by two
# already-parted models, not a bias (pooled early ratio 0.9999, whole-run log ratio +0.011 se 0.054)
FIRST_STEPS, LOSS_TOL_FIRST = 60, 0.01
# where the protocol's numbers are written (per-seed diffs, mean, sd, bound, loss ratios)
OUT = os.environ.get("MFNERF_PARITY_OUT", os.path.join(ROOT, "gpurun_out", "parity_train.json"))


def _ngp(st, cfg):
    """An NGP mirror (networks.py) holding the step's weights and the fixed occupancy."""
    class HP:
        grid, L, F, T, N_min, N_max, N_tables, rgb_channels, rgb_layers = (cfg.grid, cfg.L, cfg.F, cfg.log2_T,
                                                                           cfg.N_min, cfg.N_max, cfg.N_tables,
                                                                           cfg.rgb_width, 2)
    m = NGP(scale=cfg.scale, hparams=HP).to(st.dev)
    p = st.params
    n_net = engine.XYZ_NET_PARAMS
    with torch.no_grad():
        m.xyz_encoder.params.copy_(torch.cat([p[:n_net], p[st.off_table:st.n_params]]))
        m.rgb_net.params.copy_(p[st.off_rgb:st.off_table])
        m.density_bitfield.copy_(st.bitfield)
    return m


def _train(gpu, seed):
    """This repo's fused step on run `seed` of the protocol: (held-out PSNR, per-view PSNRs,
    {step: loss}, skipped steps)."""
    cfg = PP.config()
    st = engine.TrainStep(cfg, device=gpu, seed=PP.INIT_SEED)
    xyz0, rgb0 = PP.init_params(cfg)
    n_net = engine.XYZ_NET_PARAMS
    assert torch.equal(st.params[:n_net].cpu(), xyz0[:n_net]) and torch.equal(st.params[st.off_rgb:st.off_table].cpu(),
                                                                              rgb0)
    assert torch.equal(st.params[st.off_table:st.n_params].cpu(), xyz0[n_net:])
    st.set_occupancy(PP.density_grid())
    train, test = PP.scene()
    losses = {}
    for step in range(PP.STEPS):
        if step % PP.STEPS_PER_EPOCH == 0:
            st.set_lr(PP.lr_at(step))
        o, d, rgb = PP.batch(train, step, seed)
        b = engine.Batch(o.to(gpu), d.to(gpu), rgb.to(gpu))
        st.run(b, noise=PP.noise(step, seed).to(gpu))
        losses[step + 1] = float(st.loss_sum)
    model = _ngp(st, cfg)
    imgs, poses, dirs, _ = test
    views = []
    with torch.no_grad():
        for img, pose in zip(imgs, poses):
            o = pose[:, 3].expand(dirs.shape[0], 3).contiguous().to(gpu)
            dd = (dirs @ pose[:, :3].T).contiguous().to(gpu)
            views.append(PP.psnr(render(model, o, dd, test_time=True)["rgb"].cpu(), img))
    return sum(views) / len(views), views, losses, st.skipped_steps()


def _reference_runs():
    """The reference side's runs: parity_train.json (run 0) and parity_train_s<k>.json."""
    runs = [json.load(open(GOLDEN))]
    k = 1
    while os.path.exists(GOLDEN.replace(".json", f"_s{k}.json")):
        runs.append(json.load(open(GOLDEN.replace(".json", f"_s{k}.json"))))
        k += 1
    return runs


def _logged_steps(refs):
    """The steps whose loss both sides hold: every step when the fixtures record it (1600 batch
    losses per epoch over 8 seeds), else every LOG_EVERY-th step (80 per epoch -- then the
    per-epoch ratio carries a few percent of batch-to-batch noise)."""
    if all("loss_every_step" in r for r in refs):
        return list(range(1, PP.STEPS + 1))
    return [h["step"] for h in refs[0]["history"]]


def _reference_losses(ref, steps):
    if "loss_every_step" in ref:
        return [ref["loss_every_step"][st - 1] for st in steps]
    by = {h["step"]: h["loss"] for h in ref["history"]}
    return [by[st] for st in steps]


def test_training_psnr_matches_reference(gpu):
    """Paired runs (same seeds on both sides).  ONE run's held-out PSNR still varies from seed to
    seed (0.16 dB sd over 8 seeds on this side at this protocol, tools/parity_spread.py; 0.65 dB
    without the schedule's decay), so the check is statistical: the mean over the K >= 8 seeds of
    (ours - reference) must be within 0.2 dB, and within 0.2 dB plus two standard errors of that
    mean with that bound itself <= 0.35 dB; every run must be finite, skip no step, track the
    reference's loss curve epoch by epoch over the whole run, and match it closely over the first
    100 steps.  The numbers go to MFNERF_PARITY_OUT (JSON)."""
    refs = _reference_runs()
    assert len(refs) >= 8, "the protocol's reference side has fewer than 8 seeds"
    diffs, ours, theirs = [], [], []
    for ref in refs:
        seed = ref["protocol"].get("run_seed", 0)
        assert ref["protocol"]["steps"] == PP.STEPS and ref["protocol"]["n_rays"] == PP.N_RAYS
        assert ref["protocol"]["steps_per_epoch"] == PP.STEPS_PER_EPOCH and ref["protocol"]["n_test"] == PP.N_TEST
        got, views, losses, skipped = _train(gpu, seed)
        print(f"\nPARITY seed {seed}: held-out PSNR ours {got:.3f} reference {ref['test_psnr']:.3f} "
              f"(diff {got - ref['test_psnr']:+.3f}) skipped steps {skipped}")
        assert skipped == 0 and got == got
        diffs.append(got - ref["test_psnr"])
        steps = _logged_steps(refs)
        ours.append([losses[st] for st in steps])
        theirs.append(_reference_losses(ref, steps))
        print("PARITY_LOSSES " + json.dumps({"seed": seed, "ours": ours[-1][-10:], "reference": theirs[-1][-10:]}))
    k = len(diffs)
    mean = sum(diffs) / k
    sd = (sum((d - mean) ** 2 for d in diffs) / (k - 1)) ** 0.5
    tol = 0.2 + 2.0 * sd / k ** 0.5
    # the loss curves over the WHOLE run, epoch by epoch: every step's batch loss (the same batches
    # on both sides), pooled over the seeds and the epoch's steps
    steps = _logged_steps(refs)
    ratios = []
    for e in range(PP.EPOCHS):
        idx = [i for i, st in enumerate(steps) if e * PP.STEPS_PER_EPOCH < st <= (e + 1) * PP.STEPS_PER_EPOCH]
        if idx:
            ratios.append(sum(o[i] for o in ours for i in idx) / sum(t[i] for t in theirs for i in idx))
    early = [i for i, st in enumerate(steps) if st <= EARLY_STEPS]
    early_ratio = sum(o[i] for o in ours for i in early) / sum(t[i] for t in theirs for i in early)
    # every single step of the early window: the largest deviation and where it is (seed, step)
    devs = [(abs(o[i] / t[i] - 1), seed, steps[i]) for (o, t), seed in
            zip(zip(ours, theirs), [r["protocol"].get("run_seed", 0) for r in refs]) for i in early]
    early_dev, early_dev_seed, early_dev_step = max(devs)
    first_dev, first_dev_seed, first_dev_step = max(d for d in devs if d[2] <= FIRST_STEPS)
    # the whole run after the early window: per seed the mean log ratio per step, then over seeds
    late = [i for i, st in enumerate(steps) if st > EARLY_STEPS]
    logr = [sum(math.log(o[i] / t[i]) for i in late) / len(late) for o, t in zip(ours, theirs)]
    whole_log = sum(logr) / k
    whole_se = (sum((x - whole_log) ** 2 for x in logr) / (k - 1)) ** 0.5 / k ** 0.5
    print(f"PARITY {k} seeds: mean(ours - reference) {mean:+.3f} dB, sd {sd:.3f}, bound {tol:.3f} dB; "
          f"per-epoch loss ratio ours/reference {' '.join(f'{r:.3f}' for r in ratios)}; "
          f"steps <= {EARLY_STEPS}: pooled ratio {early_ratio:.4f}, largest single deviation {early_dev:.4f} "
          f"(seed {early_dev_seed}, step {early_dev_step}); steps <= {FIRST_STEPS}: {first_dev:.4f}; "
          f"whole run mean log ratio {whole_log:+.4f} (se {whole_se:.4f})")
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump({"protocol": {"seeds": k, "steps": PP.STEPS, "epochs": PP.EPOCHS, "n_rays": PP.N_RAYS,
                                "n_test": PP.N_TEST, "early_steps": EARLY_STEPS},
                   "seeds": [r["protocol"].get("run_seed", 0) for r in refs],
                   "psnr_ours": [d + r["test_psnr"] for d, r in zip(diffs, refs)],
                   "psnr_reference": [r["test_psnr"] for r in refs],
                   "diffs_db": diffs, "mean_db": mean, "sd_db": sd, "bound_db": tol,
                   "epoch_loss_ratios": ratios, "early_loss_ratio": early_ratio,
                   "early_max_single_deviation": early_dev,
                   "early_max_single_deviation_at": {"seed": early_dev_seed, "step": early_dev_step},
                   "first_steps": FIRST_STEPS, "first_max_single_deviation": first_dev,
                   "first_max_single_deviation_at": {"seed": first_dev_seed, "step": first_dev_step},
                   # every step of the early window, per seed (ours / reference - 1)
                   "early_deviation_per_step": [[o[i] / t[i] - 1 for i in early] for o, t in zip(ours, theirs)],
                   "whole_run_log_ratio_per_seed": logr, "whole_run_log_ratio": whole_log,
                   "whole_run_log_ratio_se": whole_se,
                   "loss_steps_pooled": len(steps),
                   # the curves themselves every LOG_EVERY steps (the file stays small)
                   "loss_steps": [st for st in steps if st % PP.LOG_EVERY == 0],
                   "loss_ours": [[o[i] for i, st in enumerate(steps) if st % PP.LOG_EVERY == 0] for o in ours],
                   "loss_reference": [[t[i] for i, st in enumerate(steps) if st % PP.LOG_EVERY == 0] for t in theirs]},
                  f, indent=1)
    assert tol <= 0.35, (diffs, tol)
    assert abs(mean) <= 0.2, (diffs, mean)
    assert abs(mean) < tol, (diffs, tol)
    assert len(ratios) == PP.EPOCHS and all(abs(r - 1) < LOSS_TOL_EPOCH for r in ratios), ratios
    assert abs(early_ratio - 1) < LOSS_TOL_EARLY, (early_ratio, early_dev)
    assert first_dev <= LOSS_TOL_FIRST, (first_dev, first_dev_seed, first_dev_step)
    assert abs(whole_log) <= WHOLE_LOG_TOL and abs(whole_log) <= WHOLE_SE_K * whole_se + 1e-3, (whole_log, whole_se)

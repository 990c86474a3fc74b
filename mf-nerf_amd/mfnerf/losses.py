"""losses.py of the reference (NeRFLoss, DistortionLoss) over the gfx950 `vren` ops."""
import torch
from torch import nn

from . import vren


class DistortionLoss(torch.autograd.Function):
    """losses.py:6-37 (Mip-NeRF 360 distortion loss, DVGO-v2 formulation) -> loss (N_rays)."""

    @staticmethod
    def forward(ctx, ws, deltas, ts, rays_a):
        loss, ws_inclusive_scan, wts_inclusive_scan = vren.distortion_loss_fw(ws, deltas, ts, rays_a)
        ctx.save_for_backward(ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a)
        return loss

    @staticmethod
    def backward(ctx, dL_dloss):
        ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a = ctx.saved_tensors
        dL_dws = vren.distortion_loss_bw(dL_dloss.contiguous(), ws_inclusive_scan, wts_inclusive_scan, ws, deltas,
                                         ts, rays_a)
        return dL_dws, None, None, None


class NeRFLoss(nn.Module):
    """losses.py:40-60: squared rgb error + lambda_opacity * (-o log o) (+ distortion if enabled)."""

    def __init__(self, lambda_opacity=1e-3, lambda_distortion=1e-3):
        super().__init__()
        self.lambda_opacity = lambda_opacity
        self.lambda_distortion = lambda_distortion

    def forward(self, results, target, **kwargs):
        d = {}
        d["rgb"] = (results["rgb"] - target["rgb"]) ** 2
        o = results["opacity"] + 1e-10
        d["opacity"] = self.lambda_opacity * (-o * torch.log(o))
        if self.lambda_distortion > 0:
            d["distortion"] = self.lambda_distortion * DistortionLoss.apply(
                results["ws"], results["deltas"], results["ts"], results["rays_a"])
        return d

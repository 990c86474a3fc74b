"""Diagnostic: field backward per-tensor error vs fp32 autograd and vs an fp16-emulating oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]
import torch
from mfnerf import field as FLD
from oracle import field_oracle as FO

dev = torch.device("cuda:0")
H = lambda t: t.half().float()

def run(N, wscale, sig_on, rgb_on, seed=5):
    g = torch.Generator().manual_seed(seed)
    feat = (torch.rand(N, 32, generator=g) - 0.5).half()
    dirs = torch.randn(N, 3, generator=g)
    px = FO.xavier_uniform_(torch.empty(3072), FO.mlp_shapes(32, 16, 64, 1), g) * wscale
    pr = FO.xavier_uniform_(torch.empty(7168), FO.mlp_shapes(32, 3, 64, 2), g) * wscale
    dsig = torch.randn(N, generator=g) * 1e-6 * sig_on
    drgb = torch.randn(N, 3, generator=g) * 1e-5 * rgb_on
    f32 = feat.float().requires_grad_(True); a = H(px).requires_grad_(True); b = H(pr).requires_grad_(True)
    W1 = a[:2048].view(64, 32); W2 = a[2048:3072].view(16, 64)
    R1 = b[:2048].view(64, 32); R2 = b[2048:6144].view(64, 64); R3 = b[6144:].view(16, 64)
    y1 = torch.relu(f32 @ W1.t()); h = y1 @ W2.t()
    sigma = torch.exp(h[:, 0])
    dn = dirs / torch.norm(dirs, dim=1, keepdim=True)
    sh = FO.sh4((dn + 1) / 2)
    r1 = torch.relu(torch.cat([sh, h], 1) @ R1.t()); r2 = torch.relu(r1 @ R2.t())
    c = torch.sigmoid(r2 @ R3.t())[:, :3]
    ((sigma * dsig).sum() + (c * drgb).sum()).backward()
    packed = FLD.pack_field_weights(px.to(dev), pr.to(dev))
    dfeat = torch.empty(N, 32, device=dev); gx = torch.zeros(3072, device=dev); gr = torch.zeros(7168, device=dev)
    ws = FLD.field_bw_workspace(N, 64, dev)
    smax = float(torch.maximum(drgb.abs().max(), (dsig * sigma.detach()).abs().max()))
    S = FLD.pow2_grad_scale(smax)
    FLD.field_bw(feat.to(dev), dirs.to(dev), N, packed, dsig.to(dev), drgb.to(dev), S, dfeat, gx, gr, ws)
    torch.cuda.synchronize()
    parts = {"dfeat": (dfeat.cpu(), f32.grad), "dW1": (gx.cpu()[:2048], a.grad[:2048]),
             "dW2": (gx.cpu()[2048:], a.grad[2048:]), "dWr1": (gr.cpu()[:2048], b.grad[:2048]),
             "dWr2": (gr.cpu()[2048:6144], b.grad[2048:6144]), "dWr3": (gr.cpu()[6144:6144 + 3 * 64], b.grad[6144:6144 + 192])}
    out = [f"N={N} w={wscale} sig={sig_on} rgb={rgb_on} S={S:g} sigmax={float(sigma.max()):.3g}"]
    for k, (got, ref) in parts.items():
        if ref.abs().max() == 0:
            out.append(f"  {k}: ref zero, got max {float(got.abs().max()):.3g}"); continue
        err = float((got - ref).abs().max() / ref.abs().max())
        cos = float(torch.nn.functional.cosine_similarity(got.flatten(), ref.flatten(), dim=0))
        ratio = float((got * ref).sum() / (ref * ref).sum())
        out.append(f"  {k}: maxrel {err:.4f} cos {cos:.6f} proj {ratio:.4f}")
    print("\n".join(out), flush=True)

for args in [(3000, 1, 0, 1), (3000, 1, 1, 0), (3000, 1, 1, 1), (3000, 3, 1, 1), (64, 1, 0, 1), (32, 1, 1, 0)]:
    run(*args)

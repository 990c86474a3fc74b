"""Kernel vs an fp16-emulating manual backward (rounding exactly where the kernel packs to f16)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mf-nerf_amd")]
import torch
from mfnerf import field as FLD
from oracle import field_oracle as FO

dev = torch.device("cuda:0")
H = lambda t: t.half().float()

def emulate(feat, dirs, px, pr, dsig, drgb, S):
    f = feat.float()
    W1 = H(px[:2048].view(64, 32)); W2 = H(px[2048:3072].view(16, 64))
    R1 = H(pr[:2048].view(64, 32)); R2 = H(pr[2048:6144].view(64, 64)); R3 = H(pr[6144:].view(16, 64))
    y1 = H(torch.relu(f @ W1.t())); h = H(y1 @ W2.t())
    dn = dirs / torch.norm(dirs, dim=1, keepdim=True)
    sh = H(FO.sh4((dn + 1) / 2))
    inp = torch.cat([sh, h], 1)
    r1 = H(torch.relu(inp @ R1.t())); r2 = H(torch.relu(r1 @ R2.t()))
    o = r2 @ R3.t(); rgb = torch.sigmoid(o[:, :3])
    dO = torch.zeros(len(f), 16); dO[:, :3] = drgb * S * rgb * (1 - rgb); dO = H(dO)
    dWr3 = dO.t() @ r2
    dr2 = H((dO @ R3) * (r2 > 0))
    dWr2 = dr2.t() @ r1
    dr1 = H((dr2 @ R2) * (r1 > 0))
    dWr1 = dr1.t() @ inp
    dinp = dr1 @ R1
    dh = dinp[:, 16:].clone(); dh[:, 0] += dsig * S * torch.exp(h[:, 0].clamp(-15, 15)); dh = H(dh)
    dW2 = dh.t() @ y1
    dy1 = H((dh @ W2) * (y1 > 0))
    dW1 = dy1.t() @ f
    dX = dy1 @ W1
    return dX / S, torch.cat([dW1.flatten(), dW2.flatten()]) / S, torch.cat([dWr1.flatten(), dWr2.flatten(), dWr3.flatten()]) / S

def run(N, wscale, sig_on, rgb_on, seed=5):
    g = torch.Generator().manual_seed(seed)
    feat = (torch.rand(N, 32, generator=g) - 0.5).half()
    dirs = torch.randn(N, 3, generator=g)
    px = FO.xavier_uniform_(torch.empty(3072), FO.mlp_shapes(32, 16, 64, 1), g) * wscale
    pr = FO.xavier_uniform_(torch.empty(7168), FO.mlp_shapes(32, 3, 64, 2), g) * wscale
    dsig = torch.randn(N, generator=g) * 1e-6 * sig_on
    drgb = torch.randn(N, 3, generator=g) * 1e-5 * rgb_on
    S = 16384.0
    eX, ex, er = emulate(feat, dirs, px, pr, dsig, drgb, S)
    packed = FLD.pack_field_weights(px.to(dev), pr.to(dev))
    dfeat = torch.empty(N, 32, device=dev); gx = torch.zeros(3072, device=dev); gr = torch.zeros(7168, device=dev)
    ws = FLD.field_bw_workspace(N, 64, dev)
    FLD.field_bw(feat.to(dev), dirs.to(dev), N, packed, dsig.to(dev), drgb.to(dev), S, dfeat, gx, gr, ws)
    torch.cuda.synchronize()
    print(f"N={N} w={wscale} sig={sig_on} rgb={rgb_on}")
    for k, got, ref in (("dX", dfeat.cpu(), eX), ("dWxyz", gx.cpu(), ex), ("dWrgb", gr.cpu(), er)):
        err = float((got - ref).abs().max() / ref.abs().max())
        cos = float(torch.nn.functional.cosine_similarity(got.flatten(), ref.flatten(), dim=0))
        print(f"  {k}: maxrel {err:.2e} cos {cos:.8f}", flush=True)

for args in [(3000, 1, 0, 1), (3000, 1, 1, 1), (3000, 3, 1, 1)]:
    run(*args)

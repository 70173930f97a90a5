"""Debug helper: fused backward intermediates vs torch fp32 autograd for one config."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from ms_amd.fused import conv_gn_bwd, conv_gn_fwd, dw_to_conv, prep_weight, prep_weight_t  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def run(H, W, cin, n, use_dmask, dev="cuda"):
    torch.manual_seed(1)
    P = H * W
    x = (torch.randn(n, P, cin, device=dev) * 0.5).to(torch.bfloat16)
    w = (torch.randn(96, cin, 3, 3, device=dev) * (1.0 / (3 * cin ** 0.5))).to(torch.bfloat16).float()
    b, g, be = torch.randn(96, device=dev) * 0.1, 1 + 0.1 * torch.randn(96, device=dev), 0.1 * torch.randn(96, device=dev)
    dmask = ((torch.rand(n, 96, device=dev) > 0.1).float() / 0.9) if use_dmask else None
    out, y, st = conv_gn_fwd(x, prep_weight(w, cin), b, g, be, H, W, dmask=dmask)
    dout = torch.randn(n, P, 96, device=dev).to(torch.bfloat16)
    dx, dz, dw, dgn = conv_gn_bwd(dout, out, y, st, g, x, H, W, wT=prep_weight_t(w) if cin == 96 else None,
                                  dmask=dmask, want_dz=True)
    # reference from the SAVED bf16 y (isolates the backward)
    yr = y.float().view(n, H, W, 96).permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    gr, ber = g.clone().requires_grad_(True), be.clone().requires_grad_(True)
    zpre = F.group_norm(yr, 6, gr, ber, eps=1e-5)
    zpre.retain_grad()
    o = torch.relu(zpre)
    if dmask is not None:
        o = o * dmask[:, :, None, None]
    o.backward(dout.float().view(n, H, W, 96).permute(0, 3, 1, 2))
    nhwc = lambda t: t.permute(0, 2, 3, 1).reshape(n, P, -1)  # noqa: E731
    dyref = nhwc(yr.grad)
    print(f"{H}x{W} cin{cin} n{n} dmask={use_dmask}: dz {rel(dz, nhwc(zpre.grad)):.4f} "
          f"dgamma {rel(dgn[0], gr.grad):.4f} dbeta {rel(dgn[1], ber.grad):.4f} dbias {rel(dgn[2], yr.grad.sum((0, 2, 3))):.4f}")
    # per-sample dz error, to find bad samples
    e = (dz.float() - nhwc(zpre.grad)).flatten(1).norm(dim=1) / nhwc(zpre.grad).flatten(1).norm(dim=1).clamp_min(1e-9)
    bad = (e > 0.02).nonzero().flatten().tolist()
    print("   bad dz samples:", bad[:20], len(bad))
    # dW from exact dy
    xr = x.float().view(n, H, W, cin).permute(0, 3, 1, 2)
    wref = torch.nn.grad.conv2d_weight(xr, (96, cin, 3, 3), yr.grad, padding=1)
    print(f"   dW {rel(dw_to_conv(dw, cin), wref):.4f}")
    if cin == 96:
        dxref = torch.nn.grad.conv2d_input(xr.shape, w, yr.grad, padding=1)
        print(f"   dx {rel(dx, nhwc(dxref)):.4f}")




def partials(H=16, W=16, cin=96, n=256, dev="cuda"):
    """Per-block GN partials (one sample per block when n <= grid) vs per-sample reference sums."""
    import ms_amd.fused as FU
    from ms_amd import _lib as L
    torch.manual_seed(1)
    P = H * W
    x = (torch.randn(n, P, cin, device=dev) * 0.5).to(torch.bfloat16)
    w = (torch.randn(96, cin, 3, 3, device=dev) * (1.0 / (3 * cin ** 0.5))).to(torch.bfloat16).float()
    b, g, be = torch.randn(96, device=dev) * 0.1, 1 + 0.1 * torch.randn(96, device=dev), 0.1 * torch.randn(96, device=dev)
    out, y, st = conv_gn_fwd(x, prep_weight(w, cin), b, g, be, H, W)
    dout = torch.randn(n, P, 96, device=dev).to(torch.bfloat16)
    FU.conv_gn_bwd(dout, out, y, st, g, x, H, W, wT=prep_weight_t(w))  # init bindings
    nws = int(FU._bwd_ws(n, H, W, cin))
    work = torch.zeros(nws, device=dev)
    dy = torch.empty(n, P, 96, dtype=torch.bfloat16, device=dev)
    dz = torch.empty_like(dy)
    dx = torch.empty(n, P, cin, dtype=torch.bfloat16, device=dev)
    dw = torch.empty(9, 96, cin, device=dev)
    dgn = torch.empty(3, 96, device=dev)
    wT = prep_weight_t(w)
    FU._check(FU._bwd(L.ptr(dout), L.ptr(out), L.ptr(y), L.ptr(st), L.ptr(g), None, L.ptr(x), L.ptr(wT), None,
                      L.ptr(dy), L.ptr(dz), L.ptr(dx), L.ptr(dw), L.ptr(dgn), L.ptr(work), nws, n, H, W, cin,
                      L.stream_ptr(torch.device(dev))))
    torch.cuda.synchronize()
    part = work[: n * 3 * 96].view(n, 3, 96)
    zr = (dout.float() * (out.float() > 0)).to(torch.bfloat16).float()  # dz
    yv = y.float().view(n, P, 6, 16)
    yh = ((yv - st[:, None, :, 0:1]) * st[:, None, :, 1:2]).view(n, P, 96)
    S1 = zr.sum(1)
    S2 = (zr * yh).sum(1)
    e1 = (part[:, 1] - S1).abs().amax(1)
    e2 = (part[:, 0] - S2).abs().amax(1)
    print("S1 max err per block (top):", e1.topk(5))
    print("S2 max err per block (top):", e2.topk(5))
    print("dz err", rel(dz, zr), "sum S1 vs dgn", rel(dgn[1], S1.sum(0)), rel(part[:, 1].sum(0), S1.sum(0)))
    print("part sample", part[0, 1, :4].tolist(), S1[0, :4].tolist())


partials()

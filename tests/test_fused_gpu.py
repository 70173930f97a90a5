"""Fused conv3x3 + GroupNorm + residual + ReLU + dropout MFMA kernel vs a
PyTorch fp32 reference of the same op on the same 16-bit-rounded inputs, for both
element types (bf16, and fp16 = the reference's autocast type).
Tolerance: |d| <= 2e-2 + 2e-2*|ref| (bf16 output rounding is 2^-8 relative; fp16's
2^-11 passes the same bounds)."""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


DT = [torch.bfloat16, torch.float16]


def _ref(x, w, b, g, be, H, W, res=None, dmask=None):
    n, p, cin = x.shape
    xin = x.float().view(n, H, W, cin).permute(0, 3, 1, 2)
    wf = w.to(x.dtype).float()
    y = F.conv2d(xin, wf[:, :cin] if wf.shape[1] >= cin else wf, b, padding=1)
    z = F.group_norm(y, 6, g, be, eps=1e-5)
    if res is not None:
        z = z + res.float().view(n, H, W, 96).permute(0, 3, 1, 2)
    z = torch.relu(z)
    if dmask is not None:
        z = z * dmask[:, :, None, None]
    to_nhwc = lambda t: t.permute(0, 2, 3, 1).reshape(n, p, 96)  # noqa: E731
    y = y.contiguous()
    mean = y.reshape(n, 6, -1).mean(-1)
    rstd = torch.rsqrt(y.reshape(n, 6, -1).var(-1, unbiased=False) + 1e-5)
    return to_nhwc(z), to_nhwc(y), torch.stack([mean, rstd], -1)


# Production sizes: one PPO minibatch per GPU at each BASELINE config --
# C2/C4 16x16 (4096 envs x 64 steps / 8 = 32,768 samples; the stem too), C3 9x9 (8192 x 64 / 8 =
# 65,536), C5 30x16 (1024 envs per GPU x 64 / 8 = 8,192). They take k_wgrad's sample-group split
# and partial buffers, k_reduce's slicing and the grid sizes that the small cases never reach.
PROD = [pytest.param(16, 16, 96, 32768, id="c2-16x16-32768"), pytest.param(16, 16, 16, 32768, id="c2-stem-32768"),
        pytest.param(9, 9, 96, 65536, id="c3-9x9-65536"), pytest.param(30, 16, 96, 8192, id="c5-30x16-8192")]


@pytest.mark.parametrize("H,W,cin,n", [(16, 16, 96, 300), (16, 16, 16, 37), (9, 9, 96, 70), (30, 16, 96, 20),
                                       (16, 30, 96, 9), (5, 7, 16, 3)] + PROD)
@pytest.mark.parametrize("with_res", [False, True])
@pytest.mark.parametrize("dt", DT)
def test_conv_gn_fwd_matches_torch(gpu, H, W, cin, n, with_res, dt):
    """The fused forward (conv + bias + GroupNorm + affine [+ residual] + ReLU [+ dropout
    scale]) and its ReLU bitmask vs a torch fp32 reference of the same op."""
    _fwd_case(gpu, H, W, cin, n, with_res, dt)


def _fwd_case(gpu, H, W, cin, n, with_res, dt):
    from ms_amd.fused import conv_gn_fwd, prep_weight
    torch.manual_seed(0)
    P = H * W
    x = (torch.randn(n, P, cin, device=gpu) * (0.5 if cin == 96 else 1.0)).to(dt)
    if cin == 16:
        x[:, :, 10:] = 0  # stem: 10 obs planes zero-padded to 16
    w = torch.randn(96, cin, 3, 3, device=gpu) * (1.0 / (3 * cin ** 0.5))
    b, g, be = torch.randn(96, device=gpu) * 0.1, 1 + 0.1 * torch.randn(96, device=gpu), 0.1 * torch.randn(96, device=gpu)
    res = torch.randn(n, P, 96, device=gpu).to(dt) if with_res else None
    dmask = ((torch.rand(n, 96, device=gpu) > 0.05).float() / 0.95) if not with_res else None
    out, y, st, rm = conv_gn_fwd(x, prep_weight(w, cin, dt), b, g, be, H, W, res=res, dmask=dmask, want_mask=True)
    assert out.dtype == dt and y.dtype == dt
    ro, ry, rst = _ref(x, w, b, g, be, H, W, res, dmask)
    torch.testing.assert_close(y.float(), ry, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(st, rst, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(out.float(), ro, atol=3e-2, rtol=2e-2)
    # the ReLU bitmask is exactly out > 0 (bit j of byte c8 = channel 8*c8 + j)
    bits = (rm.to(torch.int32)[..., None] >> torch.arange(8, device=gpu, dtype=torch.int32)) & 1
    assert torch.equal(bits.reshape(n, P, 96).bool(), out.float() > 0)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _gn(y, g, b):
    """GroupNorm(6) with the affine applied elementwise: PyTorch-ROCm's fused GroupNorm
    backward returns wrong gamma/beta gradients for batches >= 256 on this image
    (tools/gn_torch_check.py), so the reference must not use it."""
    return F.group_norm(y, 6, None, None, eps=1e-5) * g[None, :, None, None] + b[None, :, None, None]


@pytest.mark.parametrize("H,W,cin,n", [(16, 16, 96, 300), (16, 16, 16, 37), (9, 9, 96, 70), (30, 16, 96, 20),
                                       (5, 7, 16, 3), (8, 8, 96, 5), (16, 16, 96, 600)] + PROD)
@pytest.mark.parametrize("with_res", [False, True])
@pytest.mark.parametrize("dt", DT)
def test_conv_gn_bwd_matches_torch(gpu, H, W, cin, n, with_res, dt):
    """Fused backward (GroupNorm backward + dgrad + wgrad) vs torch fp32 autograd.

    Tight check: the reference starts from the SAVED bf16 conv output y (what the
    backward consumes), so every gradient must agree to relative L2 <= 1e-2 (bf16
    storage of dy / dz / dx is 2^-9 relative; all sums are f32).
    Loose check: a full fp32 recompute from x, relative L2 <= 6e-2 (ReLU-mask flips
    where z ~ 0 between bf16 and fp32 activations dominate)."""
    from ms_amd.fused import (VARIANT_BWD, VARIANT_WGRAD, conv_gn_bwd, conv_gn_fwd, dw_to_conv, kernel_variant,
                              prep_weight, prep_weight_t)
    torch.manual_seed(1)
    P = H * W
    x = (torch.randn(n, P, cin, device=gpu) * (0.5 if cin == 96 else 1.0)).to(dt)
    if cin == 16:
        x[:, :, 10:] = 0
    w = (torch.randn(96, cin, 3, 3, device=gpu) * (1.0 / (3 * cin ** 0.5))).to(dt).float()
    b, g, be = torch.randn(96, device=gpu) * 0.1, 1 + 0.1 * torch.randn(96, device=gpu), 0.1 * torch.randn(96, device=gpu)
    res = torch.randn(n, P, 96, device=gpu).to(dt) if with_res else None
    dmask = ((torch.rand(n, 96, device=gpu) > 0.1).float() / 0.9) if not with_res else None
    out, y, st, rm = conv_gn_fwd(x, prep_weight(w, cin, dt), b, g, be, H, W, res=res, dmask=dmask, want_mask=True)
    dout = torch.randn(n, P, 96, device=gpu).to(dt)
    want_dx = cin == 96
    add = torch.randn(n, P, cin, device=gpu).to(dt) if (with_res and want_dx) else None
    wT = prep_weight_t(w, dt) if want_dx else None
    # the production path: the forward's ReLU bitmask
    dx, dz, dw, dgn = conv_gn_bwd(dout, None, y, st, g, x, H, W, wT=wT, dmask=dmask, addend=add, want_dz=with_res,
                                  rmask=rm)
    assert dx is None or dx.dtype == dt
    with kernel_variant(VARIANT_BWD, 1):  # the per-sample kernel: bitmask and out give bit-identical gradients
        ref_rm = conv_gn_bwd(dout, None, y, st, g, x, H, W, wT=wT, dmask=dmask, addend=add, want_dz=with_res, rmask=rm)
        ref_out = conv_gn_bwd(dout, out, y, st, g, x, H, W, wT=wT, dmask=dmask, addend=add, want_dz=with_res)
    for a_, b_ in zip(ref_rm, ref_out):
        assert (a_ is None and b_ is None) or torch.equal(a_, b_)
    for a_, b_ in zip((dx, dz, dw, dgn), ref_rm):  # the dispatcher's choice is the per-sample kernel
        assert (a_ is None and b_ is None) or torch.equal(a_, b_)
    if cin == 96 and (H, W) == (16, 16):
        # k_wgrad (three ci-slice workgroups a sample group; compiler's / pinned LDS-read schedule):
        # the same products as k_wgrad_c96 summed in another order
        dws = []
        for wv in (1, 2):
            with kernel_variant(VARIANT_WGRAD, wv):
                got = conv_gn_bwd(dout, None, y, st, g, x, H, W, wT=wT, dmask=dmask, addend=add, want_dz=with_res,
                                  rmask=rm)
            assert _rel(got[2], dw) < 1e-5, wv
            dws.append(got[2])
        assert torch.equal(dws[0], dws[1])
        with kernel_variant(VARIANT_WGRAD, 3):  # k_wgrad_c96 (the default here) by name
            got = conv_gn_bwd(dout, None, y, st, g, x, H, W, wT=wT, dmask=dmask, addend=add, want_dz=with_res,
                              rmask=rm)
        for a_, b_ in zip(got, (dx, dz, dw, dgn)):
            assert (a_ is None and b_ is None) or torch.equal(a_, b_)
    nchw = lambda t, c: t.float().view(n, H, W, c).permute(0, 3, 1, 2).contiguous()  # noqa: E731
    nhwc = lambda t: t.permute(0, 2, 3, 1).reshape(n, P, -1)  # noqa: E731
    xr = nchw(x, cin)
    dref = nchw(dout, 96)

    relu_mask = nchw(out, 96) > 0

    def chain(yin, gr, ber, own_mask):
        z = _gn(yin, gr, ber)
        if with_res:
            z = z + nchw(res, 96)
        z.retain_grad()
        o = z * relu_mask if own_mask else torch.relu(z)
        if dmask is not None:
            o = o * dmask[:, :, None, None]
        o.backward(dref)
        return z

    # tight: from the saved y
    ys = nchw(y, 96).requires_grad_(True)
    gr, ber = g.clone().requires_grad_(True), be.clone().requires_grad_(True)
    z = chain(ys, gr, ber, True)  # the kernel's own ReLU decisions (z ~ 0 flips aside)
    wgrad = torch.nn.grad.conv2d_weight(xr, (96, cin, 3, 3), ys.grad, padding=1)
    assert _rel(dw_to_conv(dw, cin), wgrad) < 1e-2
    assert _rel(dgn[0], gr.grad) < 1e-2
    assert _rel(dgn[1], ber.grad) < 1e-2
    assert _rel(dgn[2], ys.grad.sum((0, 2, 3))) < 1e-2
    if want_dx:
        dxr = torch.nn.grad.conv2d_input(xr.shape, w, ys.grad, padding=1)
        assert _rel(dx, nhwc(dxr) + (add.float() if add is not None else 0)) < 1e-2
    if with_res:
        assert _rel(dz, nhwc(z.grad)) < 1e-2
    if n > 1000:  # production sizes: the tight check above is the parity check (the loose one
        return    # below only re-tests the ReLU-flip noise, at a large cost in fp32 convolutions)
    # loose: full fp32 recompute from x
    xq = xr.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    gr2, ber2 = g.clone().requires_grad_(True), be.clone().requires_grad_(True)
    chain(F.conv2d(xq, wr, br, padding=1), gr2, ber2, False)
    assert _rel(dw_to_conv(dw, cin), wr.grad) < 6e-2
    assert _rel(dgn[0], gr2.grad) < 6e-2
    if want_dx:
        assert _rel(dx, nhwc(xq.grad) + (add.float() if add is not None else 0)) < 6e-2


@pytest.mark.parametrize("n,P", [(300, 256), (7, 81), (3, 30), (50, 12), pytest.param(32768, 256, id="c2-32768x256"),
                                 pytest.param(65536, 81, id="c3-65536x81"), pytest.param(8192, 480, id="c5-8192x480")])
@pytest.mark.parametrize("with_mine", [True, False])
@pytest.mark.parametrize("dt", DT)
def test_heads_match_torch(gpu, n, P, with_mine, dt):
    """Policy + mine heads (csrc/msheads.hip) and the pooled features vs a torch fp32
    reference on the same bf16 features; gradients of f (policy path + pool only: the
    mine head reads f.detach()) and of every head parameter. Relative L2 <= 1e-2."""
    from ms_amd.fused import heads_apply
    torch.manual_seed(3)
    mk = lambda: torch.nn.Sequential(torch.nn.Conv2d(96, 96, 1), torch.nn.ReLU(),  # noqa: E731
                                     torch.nn.Conv2d(96, 1, 1)).to(gpu)
    pol, mine = mk(), mk()
    f = (torch.randn(n, P, 96, device=gpu) * 0.7).to(dt).requires_grad_(True)
    wl, wp, wm = torch.randn(n, P, device=gpu), torch.randn(n, 96, device=gpu), torch.randn(n, P, device=gpu)
    lp, pooled, lm = heads_apply(f, pol, mine if with_mine else None)
    loss = (lp * wl).sum() + (pooled * wp).sum() + ((lm * wm).sum() if with_mine else 0)
    loss.backward()
    got = {k: v.grad.clone() for k, v in list(pol.named_parameters()) + [("f", f)]}
    got.update({"m" + k: v.grad.clone() for k, v in mine.named_parameters()} if with_mine else {})
    for mod in (pol, mine):
        mod.zero_grad(set_to_none=True)
    fr = f.detach().float().requires_grad_(True)
    # the kernel's W1 is 16-bit (as under the reference's autocast): round it the same way
    bfw = lambda w: w + (w.detach().to(dt).float() - w.detach())  # noqa: E731  (grad flows to w)
    lin = lambda h, t: torch.nn.functional.linear(  # noqa: E731
        torch.relu(torch.nn.functional.linear(t, bfw(h[0].weight.flatten(1)), h[0].bias)), h[2].weight.flatten(1),
        h[2].bias).squeeze(-1)
    rp = lin(pol, fr)
    rpool = fr.mean(1)
    rloss = (rp * wl).sum() + (rpool * wp).sum()
    if with_mine:
        rm = lin(mine, fr.detach())
        rloss = rloss + (rm * wm).sum()
    rloss.backward()
    assert _rel(lp, rp) < 1e-2 and _rel(pooled, rpool) < 1e-3
    if with_mine:
        assert _rel(lm, rm) < 1e-2
    ref = {k: v.grad for k, v in list(pol.named_parameters()) + [("f", fr)]}
    ref.update({"m" + k: v.grad for k, v in mine.named_parameters()} if with_mine else {})
    for k in ref:
        assert _rel(got[k], ref[k]) < 1e-2, (k, _rel(got[k], ref[k]))


@pytest.mark.parametrize("n,P", [(2048, 256), (1000, 81), (9, 12)])
def test_heads_bwd_deterministic(gpu, n, P):
    """Two backward passes of the heads on the same inputs give bitwise-equal gradients (the
    per-workgroup partials are combined in a fixed order; round 4's LDS float atomics for dw2 /
    db1 were not, and the RCCL world-1 check caught it)."""
    from ms_amd.fused import heads_apply
    torch.manual_seed(5)
    mk = lambda: torch.nn.Sequential(torch.nn.Conv2d(96, 96, 1), torch.nn.ReLU(),  # noqa: E731
                                     torch.nn.Conv2d(96, 1, 1)).to(gpu)
    pol, mine = mk(), mk()
    f0 = (torch.randn(n, P, 96, device=gpu) * 0.7).to(torch.float16)
    wl, wp, wm = torch.randn(n, P, device=gpu), torch.randn(n, 96, device=gpu), torch.randn(n, P, device=gpu)
    outs = []
    for _ in range(2):
        for mod in (pol, mine):
            mod.zero_grad(set_to_none=True)
        f = f0.clone().requires_grad_(True)
        lp, pooled, lm = heads_apply(f, pol, mine)
        ((lp * wl).sum() + (pooled * wp).sum() + (lm * wm).sum()).backward()
        outs.append([f.grad.clone()] + [p.grad.clone() for p in list(pol.parameters()) + list(mine.parameters())])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("n,P", [(300, 256), (5, 1), (70, 81)])
def test_heads_bwd_c_api_null_gadd(gpu, n, P):
    """mc_heads_bwd called through the C ABI with gadd = NULL and dlm = NULL (both documented as
    optional, include/mscnn.h) equals the call with gadd = zeros and the mine rows' dl = zeros
    (gadd = NULL had selected the gadd-DMA kernel). M = 5 rows also covers the
    placeholder DMA reading in bounds."""
    from ms_amd import _lib as L
    from ms_amd import fused as F
    torch.manual_seed(9)
    F._heads_bind()
    M = n * P
    f = (torch.randn(M, 96, device=gpu) * 0.7).to(torch.float16)
    w1 = (torch.randn(192, 96, device=gpu) * 0.1).to(torch.float16)
    b1, w2 = torch.randn(192, device=gpu) * 0.1, torch.randn(192, device=gpu) * 0.1
    dlp = torch.randn(M, device=gpu)

    def call(gadd, dlm):
        out = [torch.empty_like(f), torch.empty(192, 96, device=gpu), torch.empty(192, device=gpu),
               torch.empty(192, device=gpu)]
        nws = int(F._hbws(M))
        work = torch.empty(nws, device=gpu)
        F._check(F._hb(L.ptr(f), L.ptr(dlp), L.ptr(dlm), L.ptr(w1), None, L.ptr(b1), L.ptr(w2), L.ptr(gadd), P,
                       L.ptr(out[0]), L.ptr(out[1]), L.ptr(out[2]), L.ptr(out[3]), L.ptr(work), nws, M,
                       F._dt(f), L.stream_ptr(gpu)))
        torch.cuda.synchronize()
        return out

    a = call(None, None)
    b = call(torch.zeros(n, 96, device=gpu), torch.zeros(M, device=gpu))
    for x, y, nm in zip(a, b, ("df", "dW1", "db1", "dw2")):
        assert torch.equal(x, y), nm


@pytest.mark.parametrize("n,dt", [(32768, torch.float16), (4100, torch.bfloat16), (64, torch.float16)])
def test_value_mlp_matches_autocast(gpu, n, dt):
    """fused.value_mlp (the value head's MLP with f32 split-K weight gradients): the forward is
    autocast's nn.Linear chain bitwise; the gradients match autocast's within its 16-bit
    rounding of the weight gradients (rel 2e-2 of the largest entry)."""
    from ms_amd import fused as F
    from ms_amd.models import CNNResidualPolicy
    torch.manual_seed(0)
    vh = CNNResidualPolicy(10, stem_channels=96, blocks=1, value_hidden=256).to(gpu).value_head
    g = torch.Generator(device=gpu).manual_seed(5)
    x = torch.randn(n, 96, device=gpu, generator=g)
    dv = torch.randn(n, device=gpu, generator=g)
    out = {}
    for mode in ("fused", "autocast"):
        vh.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=dt):
            v = F.value_mlp(vh, xi) if mode == "fused" else vh[6](torch.relu(vh[4](torch.relu(vh[2](xi))))).squeeze(-1)
        (v.float() * dv).sum().backward()
        out[mode] = (v.detach(), xi.grad.clone(), [p.grad.clone() for p in vh.parameters()])
    assert torch.equal(out["fused"][0], out["autocast"][0])
    for a, b in zip([out["fused"][1]] + out["fused"][2], [out["autocast"][1]] + out["autocast"][2]):
        assert a.shape == b.shape and a.dtype == b.dtype
        assert (a - b).abs().max().item() <= 2e-2 * b.abs().max().item() + 1e-6

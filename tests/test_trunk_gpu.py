"""The one-launch residual stack (csrc/mscnn_trunk.hip: mc_trunk_fwd / mc_trunk_bwd, with
mc_conv_wgrad per layer) against the per-layer fused kernels (mc_conv_gn_fwd / mc_conv_gn_bwd)
on the same inputs: the trunk features, every parameter gradient and every saved tensor are
BITWISE equal (same accumulation orders, same 16-bit roundings), at small shapes and at every
BASELINE config's per-GPU PPO minibatch (16x16 at 32,768 samples, 9x9 at 65,536, 30x16 at 8,192).
The per-layer path itself is pinned to fp32 PyTorch (tests/test_fused_gpu.py,
tests/test_fused_model_gpu.py), and through it to the reference's cnn_residual.py:7-96."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu


def _obs(n, H, W, dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    idx = torch.randint(0, 10, (n, H, W), device=dev, generator=g)
    return torch.nn.functional.one_hot(idx, 10).permute(0, 3, 1, 2).float().contiguous()


def _model(blocks, dev, seed=0):
    from ms_amd.models import CNNResidualPolicy
    torch.manual_seed(seed)
    m = CNNResidualPolicy(10, stem_channels=96, blocks=blocks, dropout=0.05, value_hidden=64).to(dev).train()
    with torch.no_grad():  # non-trivial GroupNorm affine parameters
        for mod in m.modules():
            if isinstance(mod, torch.nn.GroupNorm):
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.3, 0.3)
    return m


def _dmasks(blocks, n, dev, p=0.05):
    g = torch.Generator(device=dev).manual_seed(7)
    return [((torch.rand(n, 96, device=dev, generator=g) >= p).float() / (1.0 - p)).contiguous() for _ in range(blocks)]


def _run(m, obs, dt, dmasks, chain, grad=True):
    from ms_amd import fused as F
    H, W = obs.shape[-2:]
    with F.chain_path(chain):
        assert F.chain_ok(F.trunk_layers(m), H, W) == chain
        m.zero_grad(set_to_none=True)
        if not grad:
            with torch.no_grad():
                return F.fused_features(m, obs, dt, dmasks=dmasks), None
        f = F.fused_features(m, obs, dt, dmasks=dmasks)
        g = torch.Generator(device=obs.device).manual_seed(3)
        df = torch.randn(f.shape, device=obs.device, generator=g).to(dt)
        f.backward(df)
        return f.detach(), {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}


def _assert_same(a, b, what):
    assert a.shape == b.shape and a.dtype == b.dtype, what
    if not torch.equal(a, b):
        d = (a.float() - b.float()).abs()
        raise AssertionError(f"{what}: {int((d > 0).sum())} elements differ, max |diff| {d.max().item():.3e}")


CASES = [  # (H, W, n, blocks)
    (16, 16, 300, 2),
    (16, 16, 1, 1),
    (9, 9, 203, 2),
    (30, 16, 40, 1),
    (16, 30, 33, 1),
    (8, 8, 70, 3),
    (5, 7, 17, 2),
]


@pytest.mark.parametrize("H,W,n,blocks", CASES)
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_trunk_chain_equals_per_layer(gpu, H, W, n, blocks, dt):
    m = _model(blocks, gpu)
    obs = _obs(n, H, W, gpu)
    dms = _dmasks(blocks, n, gpu)
    fa, ga = _run(m, obs, dt, dms, chain=True)
    fb, gb = _run(m, obs, dt, dms, chain=False)
    _assert_same(fa, fb, "features")
    assert ga.keys() == gb.keys() and len(ga) == 4 * (1 + 2 * blocks)
    for k in gb:
        _assert_same(ga[k], gb[k], k)


@pytest.mark.parametrize("H,W,n,blocks", [(16, 16, 300, 2), (30, 16, 40, 2), (9, 9, 130, 1)])
def test_trunk_chain_no_grad_equals_saved(gpu, H, W, n, blocks):
    """The no-grad forward (block outputs through the workspace, nothing saved) equals the
    saving forward and the per-layer forward."""
    dt = torch.float16
    m = _model(blocks, gpu)
    obs = _obs(n, H, W, gpu)
    dms = _dmasks(blocks, n, gpu)
    f0, _ = _run(m, obs, dt, dms, chain=True, grad=False)
    f1, _ = _run(m, obs, dt, dms, chain=False, grad=False)
    f2, _ = _run(m, obs, dt, dms, chain=True, grad=True)
    _assert_same(f0, f1, "no-grad chain vs per-layer")
    _assert_same(f0, f2, "no-grad chain vs saving chain")


@pytest.mark.parametrize("H,W,n", [(16, 16, 32768), (9, 9, 65536), (30, 16, 8192)])
def test_trunk_chain_production_size(gpu, H, W, n):
    """One PPO minibatch per GPU at each BASELINE config (the shipped 5-block model, fp16 as
    the Trainer runs it, dropout masks on): chain == per-layer bitwise, features and gradients."""
    dt = torch.float16
    m = _model(5, gpu)
    obs = _obs(n, H, W, gpu)
    dms = _dmasks(5, n, gpu)
    fa, ga = _run(m, obs, dt, dms, chain=True)
    fb, gb = _run(m, obs, dt, dms, chain=False)
    _assert_same(fa, fb, "features")
    for k in gb:
        _assert_same(ga[k], gb[k], k)


@pytest.mark.parametrize("n,dmask", [(300, True), (1, False), (4100, True)])
def test_wgrad_gn_equals_wgrad_on_saved_x(gpu, n, dmask):
    """mc_conv_wgrad_gn (x recomputed from the producing layer's y, stats, GroupNorm affine and
    dropout mask) is bitwise mc_conv_wgrad on the x the per-layer forward wrote, fp16 and bf16."""
    from ms_amd import fused as F
    H = W = 16
    m = _model(1, gpu)
    conv, norm = F.trunk_layers(m)[1]  # block 0's conv1: GroupNorm + ReLU + Dropout2d, no residual
    for dt in (torch.float16, torch.bfloat16):
        g = torch.Generator(device=gpu).manual_seed(11)
        x0 = torch.randn((n, H * W, 96), device=gpu, generator=g).to(dt).contiguous()
        dm = _dmasks(1, n, gpu)[0] if dmask else None
        wt = F._packed(conv.weight, "f", dt, 96)
        x, y, st, _ = F.conv_gn_fwd(x0, wt, conv.bias, norm.weight, norm.bias, H, W, dmask=dm, save=True,
                                    eps=norm.eps, want_mask=True)
        dy = torch.randn((n, H * W, 96), device=gpu, generator=g).to(dt).contiguous()
        assert F.wgrad_gn_ok(H, W)
        a = F.conv_wgrad_gn(dy, y, st, norm, dm, H, W)
        b = F.conv_wgrad(dy, x, H, W)
        _assert_same(a, b, f"dw {dt}")


@pytest.mark.parametrize("H,W,n,grad", [(16, 16, 300, True), (16, 16, 301, False), (9, 9, 203, True),
                                        (9, 9, 131, False), (30, 16, 40, True), (5, 7, 17, False)])
def test_trunk_pooled_equals_mean(gpu, H, W, n, grad):
    """The value head's global average pool taken by the trunk kernel from the last tile on chip
    (mc_trunk_fwd_pooled; k_trunk_fwd with saves, k_trunk_fwd2 without, odd N) equals the f32
    mean of the features it wrote, within f32 summation-order rounding."""
    from ms_amd import fused as F
    m = _model(2, gpu)
    obs = _obs(n, H, W, gpu)
    with torch.set_grad_enabled(grad):
        f, pooled = F.fused_features(m, obs, torch.float16, dmasks=_dmasks(2, n, gpu), with_pooled=True)
    ref = f.detach().mean(1, dtype=torch.float32)
    assert pooled.shape == (n, 96) and pooled.dtype == torch.float32
    torch.testing.assert_close(pooled, ref, rtol=1e-5, atol=1e-5)

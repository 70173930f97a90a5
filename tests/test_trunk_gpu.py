"""The one-launch residual stack (csrc/mscnn_trunk.hip: mc_trunk_fwd / mc_trunk_bwd, with
mc_conv_wgrad per layer) against the per-layer fused kernels (mc_conv_gn_fwd / mc_conv_gn_bwd)
on the same inputs, at small shapes and at every BASELINE config's per-GPU PPO minibatch (16x16 at
32,768 samples, 9x9 at 65,536, 30x16 at 8,192).
* The saving (training) forward -- k_trunk_fwd2 on boards of <= 256 cells, k_trunk_fwd above --
  and the one-launch backward keep the per-layer kernels' accumulation orders and roundings:
  features, every parameter gradient and every saved tensor are BITWISE equal.
* The no-grad (rollout) forward on <= 256 cells, k_trunk_fwd_pp (ping-pong teams, pixel-major
  accumulators starting from the conv bias), sums the conv bias and the GroupNorm statistics in
  another f32 order: its features agree with the per-layer path to 16-bit rounding (relative L2
  bounds PP_TOL below, the measured errors x 3-4); forced onto the training forward as well
  (mc_set_variant(3, 2)) its gradients stay within PP_TOL too, and the model through it is pinned
  to fp32 PyTorch in tests/test_fused_model_gpu.py at the per-layer path's bounds.
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


def _run(m, obs, dt, dmasks, chain, grad=True, variant=0):
    from ms_amd import fused as F
    H, W = obs.shape[-2:]
    with F.chain_path(chain), F.kernel_variant(F.VARIANT_TRUNK_FWD, variant):
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


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


# k_trunk_fwd_pp vs the per-layer path, relative L2 (measured on gfx950 up to 8,191 samples: features
# <= 5.0e-4 fp16 / 2.7e-3 bf16, every parameter gradient <= 2.5e-2 fp16 / 4.4e-2 bf16, the worst
# being GroupNorm biases whose gradients are cancelling sums; the median gradient <= 3e-3)
PP_TOL = {torch.float16: dict(feat=2e-3, grad=8e-2, grad_median=1e-2),
          torch.bfloat16: dict(feat=1e-2, grad=1.5e-1, grad_median=3e-2)}


def _assert_close_pp(fa, ga, fb, gb, dt, what=""):
    tol = PP_TOL[dt]
    assert fa.shape == fb.shape and fa.dtype == fb.dtype
    assert _rel(fa, fb) <= tol["feat"], f"{what} features rel {_rel(fa, fb):.2e}"
    if ga is None:
        return
    assert ga.keys() == gb.keys()
    errs = sorted((_rel(ga[k], gb[k]), k) for k in gb)
    assert errs[-1][0] <= tol["grad"], f"{what} worst gradient {errs[-1][1]} rel {errs[-1][0]:.2e}"
    med = errs[len(errs) // 2][0]
    assert med <= tol["grad_median"], f"{what} median gradient rel {med:.2e}"


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
    """The saving forward (k_trunk_fwd2 / k_trunk_fwd) and the one-launch backward: bitwise the
    per-layer kernels."""
    m = _model(blocks, gpu)
    obs = _obs(n, H, W, gpu)
    dms = _dmasks(blocks, n, gpu)
    fa, ga = _run(m, obs, dt, dms, chain=True)
    fb, gb = _run(m, obs, dt, dms, chain=False)
    _assert_same(fa, fb, "features")
    assert ga.keys() == gb.keys() and len(ga) == 4 * (1 + 2 * blocks)
    for k in gb:
        _assert_same(ga[k], gb[k], k)


@pytest.mark.parametrize("H,W,n,blocks", CASES)
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_trunk_pp_close_to_per_layer(gpu, H, W, n, blocks, dt):
    """k_trunk_fwd_pp forced onto the saving forward (variant 2: y, statistics, ReLU bits and
    block outputs from its pixel-major epilogue) + the one-launch backward against the per-layer
    kernels: features and every gradient within PP_TOL."""
    m = _model(blocks, gpu)
    obs = _obs(n, H, W, gpu)
    dms = _dmasks(blocks, n, gpu)
    fa, ga = _run(m, obs, dt, dms, chain=True, variant=2)
    fb, gb = _run(m, obs, dt, dms, chain=False)
    assert len(ga) == 4 * (1 + 2 * blocks)
    if H * W > 256:  # k_trunk_fwd: bitwise
        _assert_same(fa, fb, "features")
    _assert_close_pp(fa, ga, fb, gb, dt, f"{H}x{W} n={n}")


@pytest.mark.parametrize("H,W,n,blocks", [(16, 16, 300, 2), (30, 16, 40, 2), (9, 9, 130, 1)])
def test_trunk_chain_no_grad_equals_saved(gpu, H, W, n, blocks):
    """The no-grad forward (block outputs through the workspace, nothing saved): with either
    forward kernel forced (variants 1 / 2) it equals that kernel's saving forward bitwise; the
    default (k_trunk_fwd_pp on <= 256 cells) is within PP_TOL of the per-layer forward, k_trunk_fwd2
    and k_trunk_fwd are bitwise equal to it."""
    dt = torch.float16
    m = _model(blocks, gpu)
    obs = _obs(n, H, W, gpu)
    dms = _dmasks(blocks, n, gpu)
    f1, _ = _run(m, obs, dt, dms, chain=False, grad=False)
    for variant in (1, 2):
        f0, _ = _run(m, obs, dt, dms, chain=True, grad=False, variant=variant)
        f2, _ = _run(m, obs, dt, dms, chain=True, grad=True, variant=variant)
        _assert_same(f0, f2, f"no-grad chain vs saving chain (variant {variant})")
        if variant == 1 or H * W > 256:
            _assert_same(f0, f1, "no-grad chain vs per-layer")
        else:
            _assert_close_pp(f0, None, f1, None, dt, "no-grad")
    fd, _ = _run(m, obs, dt, dms, chain=True, grad=False)
    _assert_same(fd, f0, "default no-grad forward vs variant 2" if H * W <= 256 else "default vs variant 2")


@pytest.mark.parametrize("H,W,n", [(16, 16, 32768), (9, 9, 65536), (30, 16, 8192)])
def test_trunk_chain_production_size(gpu, H, W, n):
    """One PPO minibatch per GPU at each BASELINE config (the shipped 5-block model, fp16 as
    the Trainer runs it, dropout masks on): the training chain == per-layer bitwise, features and
    gradients; the default no-grad forward within PP_TOL (bitwise at 30x16)."""
    dt = torch.float16
    m = _model(5, gpu)
    obs = _obs(n, H, W, gpu)
    dms = _dmasks(5, n, gpu)
    fb, gb = _run(m, obs, dt, dms, chain=False)
    fa, ga = _run(m, obs, dt, dms, chain=True)
    _assert_same(fa, fb, "features")
    for k in gb:
        _assert_same(ga[k], gb[k], k)
    del ga, gb
    fn, _ = _run(m, obs, dt, dms, chain=True, grad=False)
    if H * W > 256:
        _assert_same(fn, fb, "no-grad features")
    else:
        _assert_close_pp(fn, None, fb, None, dt, f"no-grad {H}x{W} n={n}")


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
@pytest.mark.parametrize("variant", [0, 2])
def test_trunk_pooled_equals_mean(gpu, H, W, n, grad, variant):
    """The value head's global average pool taken by the trunk kernel on chip (mc_trunk_fwd_pooled;
    k_trunk_fwd_pp: reduced from the last layer's registers, k_trunk_fwd: from the last tile; odd N)
    equals the f32 mean of the features it wrote, within f32 summation-order rounding."""
    from ms_amd import fused as F
    m = _model(2, gpu)
    obs = _obs(n, H, W, gpu)
    with torch.set_grad_enabled(grad), F.kernel_variant(F.VARIANT_TRUNK_FWD, variant):
        f, pooled = F.fused_features(m, obs, torch.float16, dmasks=_dmasks(2, n, gpu), with_pooled=True)
    ref = f.detach().mean(1, dtype=torch.float32)
    assert pooled.shape == (n, 96) and pooled.dtype == torch.float32
    torch.testing.assert_close(pooled, ref, rtol=1e-5, atol=1e-5)

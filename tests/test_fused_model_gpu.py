"""CNNResidualPolicy through the fused MFMA trunk (bf16 or fp16 autocast) vs the same
model through PyTorch fp32 ops: outputs and every parameter gradient.
Tolerance: relative L2 error <= max(4e-2, 2 x the error of PyTorch's own autocast
path of the same type; fp16 is what the reference trains with)."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _obs(n, H, W, dev):
    # one-hot planes like the env's: 0-8 revealed counts, 9 hidden
    idx = torch.randint(0, 10, (n, H, W), device=dev)
    return torch.nn.functional.one_hot(idx, 10).permute(0, 3, 1, 2).float().contiguous()


@pytest.mark.parametrize("H,W,n,blocks", [(16, 16, 300, 2), (9, 9, 64, 1), (30, 16, 40, 2)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_fused_model_matches_fp32(gpu, H, W, n, blocks, dt):
    from ms_amd.models import CNNResidualPolicy
    torch.manual_seed(0)
    m = CNNResidualPolicy(10, stem_channels=96, blocks=blocks, dropout=0.05, value_hidden=64).to(gpu).eval()
    obs = _obs(n, H, W, gpu)
    wl, wv, wm = torch.randn(n, H * W, device=gpu), torch.randn(n, device=gpu), torch.randn(n, 1, H, W, device=gpu)

    def run(fused, amp=None):
        amp = fused if amp is None else amp
        m.fused = fused
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=dt, enabled=amp):
            assert m.use_fused(obs) == fused
            lo, v, mi = m(obs, return_mine=True)
            loss = (lo.float() * wl).sum() + (v.float() * wv).sum() + (mi.float() * wm).sum()
        loss.backward()
        return lo.float(), v.float(), mi.float(), {k: p.grad.clone() for k, p in m.named_parameters()}

    lr, vr, mr, gr = run(False)
    lb, vb, mb, gb = run(False, amp=True)  # PyTorch autocast of the same type
    lf, vf, mf, gf = run(True)
    tol = lambda ref_err: max(4e-2, 2.0 * ref_err)  # noqa: E731
    for a, b, r in ((lf, lb, lr), (vf, vb, vr), (mf, mb, mr)):
        assert _rel(a, r) < tol(_rel(b, r))
    for k in gr:
        assert _rel(gf[k], gr[k]) < tol(_rel(gb[k], gr[k])), (k, _rel(gf[k], gr[k]), _rel(gb[k], gr[k]))


def test_fused_model_train_mode_dropout(gpu):
    from ms_amd.models import CNNResidualPolicy
    torch.manual_seed(0)
    m = CNNResidualPolicy(10, stem_channels=96, blocks=2, dropout=0.5, value_hidden=64).to(gpu).train()
    obs = _obs(64, 16, 16, gpu)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert m.use_fused(obs)
        lo, v = m(obs)
        (lo.float().square().mean() + v.float().square().mean()).backward()
    assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        a, _ = m(obs)
        b, _ = m(obs)
    assert not torch.equal(a, b)  # fresh Dropout2d masks per call
    m.eval()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        a, _ = m(obs)
        b, _ = m(obs)
    assert torch.equal(a, b)


def test_fused_fp16_overflow_reaches_the_grad_scaler(gpu):
    """fp16 overflow inside the fused backward (a loss scale far too large) surfaces as
    non-finite parameter gradients, so GradScaler skips the step and lowers its scale,
    as with PyTorch's own fp16 autocast path (the reference's ppo.py:25 contract)."""
    from ms_amd.models import CNNResidualPolicy
    torch.manual_seed(0)
    m = CNNResidualPolicy(10, stem_channels=96, blocks=1, dropout=0.0, value_hidden=32).to(gpu)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    obs = _obs(64, 16, 16, gpu)
    before = {k: p.detach().clone() for k, p in m.named_parameters()}
    scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 60)
    with torch.autocast("cuda", dtype=torch.float16):
        assert m.use_fused(obs)
        lo, v = m(obs)
        loss = lo.float().square().mean() + v.float().square().mean()
    scaler.scale(loss).backward()
    assert not all(torch.isfinite(p.grad).all() for p in m.stem.parameters() if p.grad is not None)
    scaler.step(opt)
    scaler.update()
    assert scaler.get_scale() < 2.0 ** 60
    for k, p in m.named_parameters():
        assert torch.equal(p.detach(), before[k]), k  # step skipped

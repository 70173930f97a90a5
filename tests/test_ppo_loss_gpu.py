"""The HIP PPO loss (csrc/msppo.hip via ms_amd/loss.py) against ms_amd/ppo.py's PyTorch ops of the
same loss (ppo.py:33-87) on the same model outputs: the loss terms and the gradients of the
scaled loss w.r.t. the policy logits, the value prediction and the belief logits.

Tolerances: f32 everywhere (fp32 path): terms rel 1e-5, gradients rel-norm 1e-5 per tensor.
Under 16-bit autocast the value gradient is rounded to the value's type and the belief-logit
gradient passes through the 16-bit casts as autocast's do: rel-norm 2e-3 there (a few 16-bit
roundings placed differently), f32 tolerances elsewhere. The G6 golden updates run through this
path too (tests/test_parity_gpu.py)."""
from __future__ import annotations

import ctypes
from types import SimpleNamespace

import pytest
import torch

pytestmark = pytest.mark.gpu


def _outputs(M, A, dev, vdt, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    logits = (torch.randn(M, A, generator=g) * 3).to(dev)
    mask = torch.rand(M, A, generator=g) < 0.7
    actions = torch.randint(0, A, (M,), generator=g)
    mask[torch.arange(M), actions] = True
    mask[0] = False  # a row whose only legal cell is the action
    mask[0, actions[0]] = True
    value = (torch.randn(M, generator=g)).to(vdt).to(dev)
    mine = (torch.randn(M, 1, A, generator=g) * 2).to(dev)
    labels = (torch.rand(M, A, generator=g) < 0.15).float()
    valid = torch.rand(M, A, generator=g) < 0.6
    if M > 1:
        valid[1] = False  # a row with no valid cell
    # old log-probs near the current ones: ratios on both sides of the clip range
    with torch.no_grad():
        lp = torch.log_softmax(logits.cpu().masked_fill(~mask, -1e9), -1)[torch.arange(M), actions]
    old = lp + torch.randn(M, generator=g) * 0.3
    batch = SimpleNamespace(obs=torch.zeros(M, 1, device=dev), action_mask=mask.to(dev), actions=actions.to(dev),
                            old_logp=old.to(dev), advantages=torch.randn(M, generator=g).to(dev),
                            values=(value.float().cpu() + torch.randn(M, generator=g) * 0.3).to(dev),
                            returns=(value.float().cpu() + torch.randn(M, generator=g)).to(dev),
                            mine_labels=labels.to(dev), mine_valid=valid.to(dev))
    return logits, value, mine, batch


def _run(fused, logits, value, mine, batch, cfg, amp, scale=1024.0):
    from ms_amd import loss as LS
    from ms_amd.ppo import ppo_losses
    lg = logits.clone().requires_grad_(True)
    v = value.clone().requires_grad_(True)
    mi = mine.clone().requires_grad_(True)

    def model(obs, return_mine=True):
        return (lg, v, mi) if return_mine else (lg, v)
    old = LS.FUSED_LOSS
    LS.FUSED_LOSS = fused
    try:
        out = ppo_losses(model, batch, cfg, amp_dtype=amp)
    finally:
        LS.FUSED_LOSS = old
    (out["loss"] * scale).backward()
    return {k: float(t) for k, t in out.items()}, lg.grad, v.grad, mi.grad


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.parametrize("A", [81, 256, 480], ids=["9x9", "16x16", "30x16"])
@pytest.mark.parametrize("amp", [None, torch.float16, torch.bfloat16], ids=["fp32", "fp16", "bf16"])
def test_fused_loss_matches_torch(gpu, A, amp):
    from ms_amd.ppo import PPOConfig
    cfg = PPOConfig(ent_coef=0.003, aux_mine_weight=0.05, aux_mine_calib_weight=0.01)
    vdt = amp or torch.float32
    logits, value, mine, batch = _outputs(2048 + 37, A, gpu, vdt, seed=A)
    ctx = torch.autocast("cuda", dtype=amp) if amp else torch.autocast("cuda", enabled=False)
    with ctx:
        f = _run(True, logits, value, mine, batch, cfg, amp)
        t = _run(False, logits, value, mine, batch, cfg, amp)
    assert set(f[0]) == set(t[0]) == {"loss", "policy_loss", "value_loss", "entropy", "aux_bce", "aux_calib"}
    for k in t[0]:
        assert f[0][k] == pytest.approx(t[0][k], rel=1e-5, abs=1e-6), k
    assert _rel(f[1], t[1]) <= 1e-5, "dlogits"
    assert f[2].dtype == t[2].dtype == vdt
    assert _rel(f[2], t[2]) <= (1e-5 if amp is None else 2e-3), "dvalue"
    assert _rel(f[3], t[3]) <= (1e-5 if amp is None else 2e-3), "dmine"
    assert float(f[1][~batch.action_mask].abs().max()) == 0.0  # masked cells get no gradient


def test_fused_loss_without_belief_terms(gpu):
    from ms_amd.ppo import PPOConfig
    cfg = PPOConfig(ent_coef=0.01)
    logits, value, mine, batch = _outputs(1000, 256, gpu, torch.float32, seed=3)
    f = _run(True, logits, value, mine, batch, cfg, None)
    t = _run(False, logits, value, mine, batch, cfg, None)
    assert set(f[0]) == set(t[0]) == {"loss", "policy_loss", "value_loss", "entropy"}
    for k in t[0]:
        assert f[0][k] == pytest.approx(t[0][k], rel=1e-5, abs=1e-6), k
    assert _rel(f[1], t[1]) <= 1e-5 and _rel(f[2], t[2]) <= 1e-5
    assert f[3] is None and t[3] is None


def test_fused_loss_deterministic(gpu):
    from ms_amd.ppo import PPOConfig
    cfg = PPOConfig(ent_coef=0.003, aux_mine_weight=0.05, aux_mine_calib_weight=0.01)
    logits, value, mine, batch = _outputs(32768, 256, gpu, torch.float16, seed=7)
    with torch.autocast("cuda", dtype=torch.float16):
        a = _run(True, logits, value, mine, batch, cfg, torch.float16)
        b = _run(True, logits, value, mine, batch, cfg, torch.float16)
    assert a[0] == b[0]
    for x, y in zip(a[1:], b[1:]):
        assert torch.equal(x, y)


def _torch_terms(logits, value, mine, b, cfg, world, counts):
    """ppo.py:33-87 in f64 from the same inputs (the data-parallel belief scale world / count)."""
    x = logits.double().masked_fill(~b.action_mask, -1e9)
    lp = torch.log_softmax(x, -1)
    r = (lp.gather(1, b.actions.view(-1, 1)).squeeze(1) - b.old_logp.double()).exp()
    A = b.advantages.double()
    pol = -torch.min(r * A, r.clamp(1 - cfg.clip_eps, 1 + cfg.clip_eps) * A).mean()
    v, V, R = value.double().view(-1), b.values.double(), b.returns.double()
    vc = V + (v - V).clamp(-cfg.clip_eps_v, cfg.clip_eps_v)
    val = 0.5 * torch.max((v - R) ** 2, (vc - R) ** 2).mean()
    ent = -(lp.exp() * lp).sum(-1).mean()
    lf, y = mine.double().reshape(b.mine_labels.shape), b.mine_labels.double()
    vm = torch.ones_like(y) if getattr(b, "mine_valid", None) is None else b.mine_valid.double()
    pos, cnt = counts[0].double(), counts[1].double()
    pw = (cnt - pos + 1e-6) / (pos + 1e-6)
    scale = world / cnt.clamp_min(1.0)
    bce = (torch.nn.functional.binary_cross_entropy_with_logits(lf, y, pos_weight=pw, reduction="none") * vm).sum() * scale
    cal = (((torch.sigmoid(lf) - y) ** 2) * vm).sum() * scale
    return [pol, val, ent, bce, cal]


@pytest.mark.parametrize("M,A,world,valid", [(1, 1, 1, False), (3, 5, 2, True), (517, 81, 4, False), (64, 512, 2, True)],
                         ids=["1x1", "3x5-world2", "517x81-world4-novalid", "64x512-world2"])
def test_fused_loss_edge_shapes_and_world(gpu, M, A, world, valid):
    """Odd shapes (one row, one action, the 512-cell maximum), no valid mask, and the data-parallel
    belief scale world / global count, against an f64 restatement: terms rel 1e-5."""
    from ms_amd.loss import ppo_loss_terms
    from ms_amd.ppo import PPOConfig
    cfg = PPOConfig(ent_coef=0.003, aux_mine_weight=0.05, aux_mine_calib_weight=0.01)
    logits, value, mine, b = _outputs(M, A, gpu, torch.float32, seed=M + A)
    if not valid:
        b.mine_valid = None
    vm = torch.ones_like(b.mine_labels) if b.mine_valid is None else b.mine_valid.float()
    counts = torch.stack([(b.mine_labels * vm).sum(), vm.sum()]) * 1.5  # a "global" count (other ranks)
    t = ppo_loss_terms(logits, value, mine, b, cfg, counts, world, None)
    ref = _torch_terms(logits, value, mine, b, cfg, world, counts)
    for k in range(5):
        assert float(t[k]) == pytest.approx(float(ref[k]), rel=1e-5, abs=1e-6), k
    w = [1.0, cfg.vf_coef, -cfg.ent_coef, cfg.aux_mine_weight, cfg.aux_mine_calib_weight]
    assert float(t[5]) == pytest.approx(sum(wk * float(rk) for wk, rk in zip(w, ref)), rel=1e-5, abs=1e-6)


def test_ppo_loss_c_api_rejects_bad_arguments(gpu):
    from ms_amd import _lib as L
    from ms_amd.loss import _Args, _bind
    _bind()
    lib = L.load()
    f = lib.mc_ppo_loss_fwd
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.POINTER(_Args), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    out = torch.empty(8, device=gpu)
    work = torch.empty(1 << 16, device=gpu)
    a = _Args()  # every pointer NULL
    a.M, a.A = 4, 16
    assert f(ctypes.byref(a), out.data_ptr(), work.data_ptr(), work.numel(), None) == 1  # MS_EINVAL
    lib.mc_last_error.restype = ctypes.c_char_p
    assert b"bad argument" in lib.mc_last_error()
    assert f(None, out.data_ptr(), work.data_ptr(), work.numel(), None) == 1

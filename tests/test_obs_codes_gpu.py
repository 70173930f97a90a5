"""Observation codes (the Trainer's rollout-buffer layout, ms_amd.fused.obs_encode /
codes_to_nhwc, csrc/mscnn.hip): one byte per cell instead of the f32 one-hot planes.

The encoding must be exact for every obs the env writes (env.py:172-192, including fresh
boards whose obs is all zero and every count plane 0..8), the stem input expanded from
codes must equal the one built from the f32 obs, a rollout on codes must equal the f32 run
bit for bit, and a Trainer update on codes must equal the f32 one (its rollout bitwise, its
parameter step to 1e-2)."""
from __future__ import annotations

import os

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _nhwc_ref(obs: torch.Tensor, dtype) -> torch.Tensor:
    n, c, h, w = obs.shape
    x = obs.permute(0, 2, 3, 1).reshape(n, h * w, c)
    return torch.nn.functional.pad(x, (0, 16 - c)).to(dtype)


def _env_obs(gpu, H, W, K, N, steps, seed):
    """Obs after `steps` uniform-valid steps (mix of fresh, early and late boards)."""
    from ms_amd import EnvConfig, VecMinesweeper
    vec = VecMinesweeper(N, EnvConfig(H=H, W=W, mine_count=K), seed=seed, device=gpu)
    batch = vec.reset()
    for t in range(steps):
        batch, _, _, _ = vec.step(vec.tape_actions(t, 0))
    return batch["obs"].contiguous()


@pytest.mark.parametrize("H,W,K", [(16, 16, 40), (9, 9, 10), (30, 16, 99), (16, 30, 99), (5, 7, 3)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_obs_codes_roundtrip(gpu, H, W, K, dt):
    from ms_amd.fused import codes_to_nhwc, codes_to_obs, obs_encode, obs_to_nhwc
    obs = _env_obs(gpu, H, W, K, 777, 9, seed=11)
    n = obs.shape[0]
    # every plane occurs (revealed cells with 0..several adjacent mines, hidden cells)
    assert float(obs[:, 0].sum()) > 0 and float(obs[:, 1].sum()) > 0 and float(obs[:, 2].sum()) > 0
    codes = torch.full((n, H, W), 255, dtype=torch.uint8, device=gpu)
    x_enc = obs_encode(obs, codes, want_nhwc=True, dtype=dt)
    assert int(codes.max()) <= 9
    assert torch.equal(codes_to_obs(codes), obs)
    ref = _nhwc_ref(obs, dt)
    assert torch.equal(x_enc, ref)
    assert torch.equal(codes_to_nhwc(codes, 16, dt), ref)
    assert torch.equal(obs_to_nhwc(obs, 16, dt), ref)
    assert torch.equal(obs_to_nhwc(codes, 16, dt), ref)
    # codes only (no stem input) and a board count that leaves a partial last block
    c2 = torch.zeros((n - 5, H, W), dtype=torch.uint8, device=gpu)
    assert obs_encode(obs[5:].contiguous(), c2) is None
    assert torch.equal(c2, codes[5:])


@pytest.mark.parametrize("H,W,K,late", [(16, 16, 40, False), (9, 9, 10, False), (30, 16, 99, False),
                                        (5, 7, 3, False), (16, 16, 40, True), (9, 9, 10, True)])
def test_step_codes_equals_encoded_obs(gpu, H, W, K, late):
    """ms_step_codes (the env writing the buffer's cell codes itself) against ms_step + obs_encode
    on twin handles: codes, mask, rewards, dones and the RNG states stay equal step for step,
    auto-resets and late-start resets (the k_late emit) included."""
    from ms_amd import EnvConfig, VecMinesweeper
    from ms_amd.fused import obs_encode
    N = 301
    cfg = {"prob": 0.5, "min_hidden": 5, "max_hidden": H * W // 2} if late else None
    vs = [VecMinesweeper(N, EnvConfig(H=H, W=W, mine_count=K), seed=5, device=gpu, late_start_cfg=cfg)
          for _ in range(2)]
    for v in vs:
        v.reset()
    for t in range(40):
        a = vs[0].tape_actions(t, t % 2)
        b0, r0, d0, _ = vs[0].step(a)
        ref = torch.empty((N, H, W), dtype=torch.uint8, device=gpu)
        obs_encode(b0["obs"].contiguous(), ref)
        codes = torch.full((N, H, W), 77, dtype=torch.uint8, device=gpu)
        out = {"codes": codes, "action_mask": torch.empty((N, H * W), dtype=torch.bool, device=gpu),
               "rewards": torch.empty(N, dtype=torch.float32, device=gpu),
               "dones": torch.empty(N, dtype=torch.bool, device=gpu)}
        vs[1].step(a, out=out)
        assert torch.equal(codes, ref), t
        assert torch.equal(out["action_mask"], b0["action_mask"]) and torch.equal(out["rewards"], r0)
        assert torch.equal(out["dones"], d0)
    import numpy as np
    assert np.array_equal(np.asarray(vs[0].rng_state()), np.asarray(vs[1].rng_state()))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_obs_to_nhwc_any_f32_input(gpu, dt):
    """The fused model's input conversion of an f32 obs is the cast of its values, whatever they
    are (a caller's own planes need not be one-hot)."""
    from ms_amd.fused import obs_to_nhwc
    g = torch.Generator(device=gpu).manual_seed(3)
    obs = torch.randn((37, 10, 9, 7), device=gpu, generator=g)
    assert torch.equal(obs_to_nhwc(obs, 16, dt), _nhwc_ref(obs, dt))
    idx = torch.randint(0, 10, (37, 9, 7), device=gpu, generator=g)
    oh = torch.nn.functional.one_hot(idx, 10).permute(0, 3, 1, 2).float().contiguous()
    assert torch.equal(obs_to_nhwc(oh, 16, dt), _nhwc_ref(oh, dt))


def test_obs_encode_rejects_bad_arguments(gpu):
    from ms_amd import _lib as L
    from ms_amd.fused import obs_encode
    obs = torch.zeros((4, 10, 3, 3), device=gpu)
    with pytest.raises(AssertionError):
        obs_encode(obs, torch.zeros((4, 3, 3), dtype=torch.int32, device=gpu))
    lib = L.load()
    assert lib.mc_obs_encode(None, None, None, 0, 9, 16, 0, None) != 0


def _small_model(gpu, H, W, seed=0):
    from ms_amd.models import build_model
    torch.manual_seed(seed)
    return build_model("cnn_residual", obs_shape=(10, H, W),
                       model_cfg=dict(stem_channels=96, blocks=1, dropout=0.05, value_hidden=32)).to(gpu)


@pytest.mark.parametrize("amp", [torch.float16, None])
def test_collect_rollout_codes_equals_f32(gpu, amp):
    """Same envs, model and sampler seeds: the codes buffer decodes to the f32 buffer and every
    stored quantity (actions, logp, values, rewards, dones, labels) is bitwise equal (fused fp16
    trunk, and the fp32 PyTorch chain fed by codes_to_obs)."""
    from ms_amd import EnvConfig, VecMinesweeper
    from ms_amd.fused import codes_to_obs
    from ms_amd.rollout import collect_rollout
    H, W, K, N, T = 16, 16, 40, 256, 6
    bufs = {}
    for codes in (False, True):
        vec = VecMinesweeper(N, EnvConfig(H=H, W=W, mine_count=K), seed=5, device=gpu)
        model = _small_model(gpu, H, W).train()
        buf, aux = collect_rollout(vec, model, T, gpu, aux_mine_weight=0.05, amp_dtype=amp, sample_seed=3,
                                   obs_codes=codes)
        assert buf.obs_codes == codes
        bufs[codes] = (buf, aux)
    (bf, af), (bc, ac) = bufs[False], bufs[True]
    assert bc.obs.dtype == torch.uint8 and bc.obs.shape == (N * T, H, W)
    assert torch.equal(codes_to_obs(bc.obs), bf.obs)
    for name in ("action_mask", "actions", "logp", "values", "rewards", "dones", "mine_labels", "mine_valid"):
        assert torch.equal(getattr(bc, name), getattr(bf, name)), name
    assert torch.equal(ac["last_obs"], af["last_obs"]) and torch.equal(ac["last_values"], af["last_values"])


def test_trainer_update_codes_equals_f32(gpu):
    """One Trainer update (rollout + GAE + minibatch updates, fused fp16 + GradScaler) with the
    codes buffer: the rollout it stores is bitwise the f32-buffer run's (decoded obs, actions,
    logp, values, rewards, dones, labels, advantages), and the parameter step agrees per tensor
    to 1e-2 relative L2. (The update itself is not bitwise reproducible run to run: the value
    head's hipBLASLt weight-gradient GEMMs may split K; an input mismatch would show as an
    O(1) difference.)"""
    from ms_amd.fused import codes_to_obs
    from ms_amd.train import Trainer, load_config
    out = {}
    for codes in (False, True):
        cfg, env_d, model_d, extras = load_config(os.path.join(ROOT, "configs", "16x16x40_medium.yaml"))
        cfg.num_envs, cfg.steps_per_env, cfg.mini_batches, cfg.ppo_epochs = 128, 8, 2, 1
        tr = Trainer(cfg, env_d, dict(model_d, blocks=1, value_hidden=32), extras, seed=0, amp="fp16",
                     device=gpu, obs_codes=codes)
        p0 = [p.detach().clone() for p in tr.model.parameters()]
        st = tr.update(0)
        assert all(torch.isfinite(torch.tensor(v)) for v in st.values()), st
        assert tr.buffer.obs_codes == codes
        out[codes] = (p0, [p.detach().clone() for p in tr.model.parameters()], tr.buffer)
    (i0, p0, bf), (i1, p1, bc) = out[False], out[True]
    assert all(torch.equal(a, b) for a, b in zip(i0, i1))
    assert torch.equal(codes_to_obs(bc.obs), bf.obs)
    for name in ("action_mask", "actions", "logp", "values", "rewards", "dones", "advantages", "returns",
                 "mine_labels", "mine_valid"):
        assert torch.equal(getattr(bc, name), getattr(bf, name)), name
    for a0, a, b in zip(i0, p0, p1):
        da, db = (a - a0).float(), (b - a0).float()
        assert float((da - db).norm()) <= 1e-2 * float(da.norm()) + 1e-9

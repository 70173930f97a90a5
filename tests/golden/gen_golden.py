"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

Run in the build container only (the reference does not exist on the GPU box):

    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

It imports yakvrz/minesweeper-ppo read-only and writes data-only ``.npz``
files (inputs and expected outputs). Nothing from the reference's source is
copied; the fixtures are what its code computes on numpy 2.2.6 / torch 2.10
(CPU) in this container. The tests only read the ``.npz`` files.

Fixtures
  G1 seeds_*.npz      per-env seed lists + RNG states (env.py:393-395, 49)
  G2 place_*.npz      first-click mine placement + counts + post-draw RNG state
                      (env.py:280-335) for corner/edge/interior clicks
  G3 traj_*.npz       VecMinesweeper trajectories under the shared action tape
                      (env.py:468-511), incl. late start (env.py:416-466)
  G4 gae.npz          RolloutBuffer.compute_gae (buffers.py:78-94)
  G5 model_*.npz      CNNResidualPolicy / CNNPolicy eval-mode fp32 outputs
                      (models/cnn_residual.py:30-96, models/cnn.py)
  G6 ppo.npz          one ppo_update on the small model (ppo.py:23-119)
     ppo_full_16x16.npz one ppo_update on the shipped 96x5 model, with its fp32 and
                      float64 gradients
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
M64 = (1 << 64) - 1

import torch  # noqa: E402

from minesweeper.env import EnvConfig, MinesweeperEnv, VecMinesweeper  # noqa: E402
from minesweeper.buffers import RolloutBuffer  # noqa: E402
from minesweeper.models import build_model  # noqa: E402
from minesweeper.ppo import PPOConfig, ppo_update  # noqa: E402


def splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def tape_action(g: int, t: int, mode: int, mask_row: np.ndarray, mine_row: np.ndarray) -> int:
    """SURVEY.md §8d action tape (same rule as include/msenv.h ms_tape_actions)."""
    x = splitmix64(0xC0FFEE ^ ((g << 32) & M64) ^ t)
    valid = np.flatnonzero(mask_row)
    safe = np.flatnonzero(mask_row & ~mine_row)
    if mode == 1 and (x & 0xFFFF) < 65208 and len(safe) > 0:
        return int(safe[(x >> 16) % len(safe)])
    if len(valid) == 0:
        return 0
    sel = (x >> 16) if mode == 1 else x
    return int(valid[sel % len(valid)])


def rng_state(gen: np.random.Generator) -> np.ndarray:
    s = gen.bit_generator.state
    st, inc = s["state"]["state"], s["state"]["inc"]
    return np.array([st >> 64, st & M64, inc >> 64, inc & M64, s["has_uint32"], s["uinteger"]],
                    dtype=np.uint64)


def obs_codes(obs: np.ndarray) -> np.ndarray:
    """[N,10,H,W] f32 one-hot obs -> [N,H*W] u8 code (0 hidden, 1+count revealed).
    A revealed cell before the first click (never happens) would give code 1 with
    no count plane; planes are checked to be one-hot per revealed cell."""
    N, C, H, W = obs.shape
    rev = obs[:, 0] > 0
    cnt = np.argmax(obs[:, 1:], axis=1)
    has = obs[:, 1:].sum(axis=1)
    assert np.all(has[rev] <= 1) and np.all(has[~rev] == 0)
    code = np.where(rev, 1 + cnt * (has > 0), 0).astype(np.uint8)
    # 255 marks "revealed but no count plane" so the fixture stays exact
    code = np.where(rev & (has == 0), 255, code).astype(np.uint8)
    return code.reshape(N, H * W)


def gen_seeds():
    for base in (0, 1, 12345):
        g = np.random.default_rng(base)
        seeds = g.integers(0, 2**31 - 1, size=64, dtype=np.int64)
        after = rng_state(g)
        env_states = np.stack([rng_state(np.random.default_rng(int(s))) for s in seeds])
        np.savez_compressed(os.path.join(HERE, f"seeds_{base}.npz"), base=np.int64(base),
                            seeds=seeds, base_state_after=after, env_states=env_states)


def gen_place():
    cases = [(16, 16, 40, True), (9, 9, 10, True), (30, 16, 99, True), (16, 30, 99, True),
             (8, 8, 10, False), (4, 4, 15, True), (5, 7, 20, True)]
    for H, W, K, gsafe in cases:
        clicks = [(0, 0), (0, W // 2), (H // 2, W // 2), (H - 1, W - 1), (H // 2, 0)]
        mines, counts, states, seeds, cl = [], [], [], [], []
        for seed in (0, 3, 99, 2**31 - 2):
            for (r, c) in clicks:
                env = MinesweeperEnv(EnvConfig(H=H, W=W, mine_count=K,
                                               guarantee_safe_neighborhood=gsafe), seed=seed)
                env._place_mines_safe((r, c))
                mines.append(env.mine_mask.reshape(-1).copy())
                counts.append(env.adjacent_counts.reshape(-1).copy())
                states.append(rng_state(env.rng))
                seeds.append(seed)
                cl.append((r, c))
        np.savez_compressed(os.path.join(HERE, f"place_{H}x{W}x{K}_{int(gsafe)}.npz"),
                            H=H, W=W, K=K, guarantee=int(gsafe), seeds=np.array(seeds, np.int64),
                            clicks=np.array(cl, np.int64), mines=np.array(mines, bool),
                            counts=np.array(counts, np.uint8), states=np.array(states, np.uint64))


OUT_CODE = {None: 0, "win": 1, "loss": 2}


def gen_traj(H, W, K, N, T, mode, seed, late=None, tag=""):
    cfg = EnvConfig(H=H, W=W, mine_count=K)
    vec = VecMinesweeper(N, cfg, seed=seed, late_start_cfg=late,
                         late_start_seed=(seed + 1) if late else None)
    d = vec.reset()
    A = H * W
    reset_codes = obs_codes(d["obs"])
    acts = np.zeros((T, N), np.int64)
    rew = np.zeros((T, N), np.float32)
    done = np.zeros((T, N), bool)
    outc = np.zeros((T, N), np.int8)
    stp = np.zeros((T, N), np.int32)
    lnew = np.zeros((T, N), np.int32)
    frac = np.zeros((T, N), np.float64)
    codes = np.zeros((T, N, A), np.uint8)
    mines = np.zeros((T, N, (A + 7) // 8), np.uint8)
    mask = d["action_mask"]
    for t in range(T):
        a = np.array([tape_action(i, t, mode, mask[i], vec.envs[i].mine_mask.reshape(-1))
                      for i in range(N)], np.int64)
        acts[t] = a
        d, r, dn, info = vec.step(a)
        rew[t] = r
        done[t] = dn
        outc[t] = [OUT_CODE[o] for o in info["outcome"]]
        stp[t] = [x["step"] for x in info["aux"]]
        lnew[t] = [x["last_new_reveals"] for x in info["aux"]]
        frac[t] = [x["revealed_frac"] for x in info["aux"]]
        codes[t] = obs_codes(d["obs"])
        assert np.array_equal(d["action_mask"], ~(d["obs"][:, 0] > 0).reshape(N, A))
        mines[t] = np.packbits(np.stack([e.mine_mask.reshape(-1) for e in vec.envs]), axis=1)
        mask = d["action_mask"]
    end_states = np.stack([rng_state(e.rng) for e in vec.envs])
    name = f"traj_{H}x{W}x{K}_m{mode}{tag}.npz"
    extra = {}
    if late:
        extra = dict(late_prob=late["prob"], late_min=late["min_hidden"],
                     late_max=late["max_hidden"], late_state=rng_state(vec._late_rng))
    np.savez_compressed(os.path.join(HERE, name), H=H, W=W, K=K, N=N, T=T, mode=mode, seed=seed,
                        reset_codes=reset_codes, actions=acts, rewards=rew, dones=done,
                        outcome=outc, step=stp, last_new=lnew, frac=frac, codes=codes,
                        mines=mines, end_states=end_states, **extra)
    wins = int((outc == 1).sum())
    losses = int((outc == 2).sum())
    print(f"{name}: wins={wins} losses={losses}", flush=True)


def gen_gae():
    g = torch.Generator().manual_seed(0)
    T, N = 64, 32
    buf = RolloutBuffer(num_envs=N, steps=T, obs_shape=(10, 4, 4), action_dim=16,
                        device=torch.device("cpu"))
    buf.rewards.copy_(torch.randn(T * N, generator=g))
    buf.values.copy_(torch.randn(T * N, generator=g))
    buf.dones.copy_(torch.rand(T * N, generator=g) < 0.1)
    last = torch.randn(N, generator=g)
    buf.compute_gae(last, gamma=0.995, lam=0.95)
    np.savez_compressed(os.path.join(HERE, "gae.npz"), T=T, N=N, gamma=0.995, lam=0.95,
                        rewards=buf.rewards.numpy(), values=buf.values.numpy(),
                        dones=buf.dones.numpy(), last_values=last.numpy(),
                        advantages=buf.advantages.numpy(), returns=buf.returns.numpy())


def _sd_to_npz(sd):
    return {"w::" + k: v.detach().cpu().numpy().copy() for k, v in sd.items()}


def _sha(model):
    h = hashlib.sha256()
    for k, v in model.state_dict().items():
        h.update(k.encode())
        h.update(v.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def _sha_sd(npz_sd):
    """sha256 over an _sd_to_npz dict (the initial weights are re-made by seeded init)."""
    h = hashlib.sha256()
    for k, v in npz_sd.items():
        h.update(k[3:].encode())
        h.update(np.ascontiguousarray(v).tobytes())
    return h.hexdigest()


def _rand_obs(n, H, W, seed):
    rng = np.random.default_rng(seed)
    obs = np.zeros((n, 10, H, W), np.float32)
    rev = rng.random((n, H, W)) < 0.4
    cnt = rng.integers(0, 9, size=(n, H, W))
    obs[:, 0] = rev
    for k in range(9):
        obs[:, 1 + k] = rev & (cnt == k)
    return obs


def gen_model():
    torch.set_float32_matmul_precision("highest")
    # small config with explicit weights
    torch.manual_seed(1)
    small = build_model("cnn_residual", obs_shape=(10, 16, 16),
                        model_cfg=dict(stem_channels=16, blocks=2, dropout=0.05, value_hidden=32)).eval()
    obs = torch.from_numpy(_rand_obs(16, 16, 16, 5))
    with torch.no_grad():
        lg, val, mine = small(obs, return_mine=True)
    np.savez_compressed(os.path.join(HERE, "model_small.npz"), obs=obs.numpy(), logits=lg.numpy(),
                        value=val.numpy(), mine=mine.numpy(), **_sd_to_npz(small.state_dict()))
    # full shipped config (configs/training/16x16x40_medium.yaml) at manual_seed(0)
    for (H, W) in ((16, 16), (9, 9), (30, 16)):
        torch.manual_seed(0)
        full = build_model("cnn_residual", obs_shape=(10, H, W),
                           model_cfg=dict(stem_channels=96, blocks=5, dropout=0.05, value_hidden=256)).eval()
        obs = torch.from_numpy(_rand_obs(8, H, W, 6))
        with torch.no_grad():
            lg, val, mine = full(obs, return_mine=True)
        np.savez_compressed(os.path.join(HERE, f"model_full_{H}x{W}.npz"), obs=obs.numpy(),
                            logits=lg.numpy(), value=val.numpy(), mine=mine.numpy(),
                            sha256=np.bytes_(_sha(full)),
                            n_params=sum(p.numel() for p in full.parameters()))
    torch.manual_seed(0)
    cnn = build_model("cnn", obs_shape=(10, 9, 9), model_cfg=dict(hidden=64)).eval()
    obs = torch.from_numpy(_rand_obs(8, 9, 9, 7))
    with torch.no_grad():
        lg, val, mine = cnn(obs, return_mine=True)
    np.savez_compressed(os.path.join(HERE, "model_cnn_9x9.npz"), obs=obs.numpy(), logits=lg.numpy(),
                        value=val.numpy(), mine=mine.numpy(), sha256=np.bytes_(_sha(cnn)))


def gen_ppo():
    torch.set_float32_matmul_precision("highest")
    torch.manual_seed(2)
    model = build_model("cnn_residual", obs_shape=(10, 8, 8),
                        model_cfg=dict(stem_channels=16, blocks=2, dropout=0.0, value_hidden=32))
    init = _sd_to_npz(model.state_dict())
    opt = torch.optim.AdamW(model.parameters(), lr=3e-4)
    B, A = 64, 64
    g = torch.Generator().manual_seed(3)
    obs = torch.from_numpy(_rand_obs(B, 8, 8, 8))
    mask = torch.rand(B, A, generator=g) < 0.7
    mask[:, 0] = True
    actions = torch.multinomial(mask.float(), 1, generator=g).squeeze(1)
    old_logp = -torch.rand(B, generator=g) * 4
    values = torch.randn(B, generator=g)
    adv = torch.randn(B, generator=g)
    rets = values + adv
    labels = (torch.rand(B, 8, 8, generator=g) < 0.2).float()
    valid = torch.rand(B, 8, 8, generator=g) < 0.6
    batch = type("Batch", (), dict(obs=obs, action_mask=mask, actions=actions, old_logp=old_logp,
                                   values=values, advantages=adv, returns=rets,
                                   mine_labels=labels, mine_valid=valid))
    cfg = PPOConfig(ent_coef=0.003, aux_mine_weight=0.05, aux_mine_calib_weight=0.01)
    stats = ppo_update(model, opt, batch, cfg, scaler=None)
    post = {"post::" + k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
    np.savez_compressed(os.path.join(HERE, "ppo.npz"), obs=obs.numpy(), mask=mask.numpy(),
                        actions=actions.numpy(), old_logp=old_logp.numpy(), values=values.numpy(),
                        advantages=adv.numpy(), returns=rets.numpy(), mine_labels=labels.numpy(),
                        mine_valid=valid.numpy(), stat_names=np.array(sorted(stats)),
                        stat_values=np.array([stats[k] for k in sorted(stats)]), **init, **post)


def gen_ppo_full():
    """G6-full: one ppo_update of the SHIPPED model (96 ch x 5 blocks, seeded init at
    manual_seed(0), dropout 0 so train mode is deterministic) on 64 16x16 samples, fp32,
    no scaler. old_logp / values are the model's own outputs plus small noise (as in a
    first PPO epoch), so no sample sits at a ratio / value clip boundary and the gradient
    is a smooth function of the forward pass. Records the clipped gradients the optimizer
    stepped on (fp32) and the same update run in float64 ("grad64::", the rounding-free
    truth the fp32 errors are measured against)."""
    torch.set_float32_matmul_precision("highest")
    H = W = 16
    A = H * W
    B = 64
    g = torch.Generator().manual_seed(13)
    obs = torch.from_numpy(_rand_obs(B, H, W, 14))
    mask = (obs[:, 0] == 0).reshape(B, A)
    mask[:, 0] = True
    actions = torch.multinomial(mask.float(), 1, generator=g).squeeze(1)
    labels = (torch.rand(B, H, W, generator=g) < 0.15).float()
    valid = mask.reshape(B, H, W) & (torch.rand(B, H, W, generator=g) < 0.9)
    n_logp = (torch.rand(B, generator=g) - 0.5) * 0.1
    n_val = (torch.rand(B, generator=g) - 0.5) * 0.1
    adv = torch.randn(B, generator=g)
    cfg = PPOConfig(ent_coef=0.003, aux_mine_weight=0.05, aux_mine_calib_weight=0.01)

    def make(dtype):
        torch.manual_seed(0)
        m = build_model("cnn_residual", obs_shape=(10, H, W),
                        model_cfg=dict(stem_channels=96, blocks=5, dropout=0.0, value_hidden=256))
        return m.to(dtype)

    model = make(torch.float32)
    init = _sd_to_npz(model.state_dict())
    with torch.no_grad():
        lg, v = model(obs)
        lp = torch.log_softmax(lg.masked_fill(~mask, -1e9), -1).gather(1, actions[:, None]).squeeze(1)
    old_logp = (lp + n_logp).float()
    values = (v.view(-1) + n_val).float()
    rets = values + adv
    out = {}
    for tag, dtype in (("", torch.float32), ("64", torch.float64)):
        m = model if dtype == torch.float32 else make(dtype)
        opt = torch.optim.AdamW(m.parameters(), lr=3e-4)
        grads = {}
        step0 = opt.step

        def step_and_record(*a, _m=m, _g=grads, _s=step0, **k):
            for n, p in _m.named_parameters():
                _g[n] = p.grad.detach().float().numpy().copy()
            return _s(*a, **k)
        opt.step = step_and_record
        c = lambda t: t.to(dtype) if t.is_floating_point() else t  # noqa: E731
        batch = type("Batch", (), dict(obs=c(obs), action_mask=mask, actions=actions, old_logp=c(old_logp),
                                       values=c(values), advantages=c(adv), returns=c(rets),
                                       mine_labels=c(labels), mine_valid=valid))
        stats = ppo_update(m, opt, batch, cfg, scaler=None)
        for n, a in grads.items():
            out[f"grad{tag}::" + n] = a
        if tag == "":
            out.update({"post::" + k: v.detach().numpy().copy() for k, v in m.state_dict().items()})
            out["stat_names"] = np.array(sorted(stats))
            out["stat_values"] = np.array([stats[k] for k in sorted(stats)])
        else:
            out["stat_values64"] = np.array([stats[k] for k in sorted(stats)])
    np.savez_compressed(os.path.join(HERE, "ppo_full_16x16.npz"), obs=obs.numpy(), mask=mask.numpy(),
                        actions=actions.numpy(), old_logp=old_logp.numpy(), values=values.numpy(),
                        advantages=adv.numpy(), returns=rets.numpy(), mine_labels=labels.numpy(),
                        mine_valid=valid.numpy(), init_sha256=np.bytes_(_sha_sd(init)), **out)


def main():
    if sys.argv[1:] == ["ppo_full"]:
        gen_ppo_full()
        return
    import minesweeper.env as E
    assert not E.HAS_ENV_NUMBA, "fixtures are defined against the BFS path; numba absent here"
    print("numpy", np.__version__, "torch", torch.__version__, file=sys.stderr)
    gen_seeds()
    gen_place()
    for (H, W, K) in ((16, 16, 40), (9, 9, 10), (16, 30, 99), (30, 16, 99), (8, 8, 10), (4, 4, 15)):
        for mode in (0, 1):
            gen_traj(H, W, K, N=16, T=200, mode=mode, seed=0)
    late = dict(prob=0.5, min_hidden=5, max_hidden=20)
    gen_traj(8, 8, 10, N=16, T=120, mode=1, seed=4, late=late, tag="_late")
    gen_traj(16, 16, 40, N=8, T=120, mode=1, seed=9, late=dict(prob=0.7, min_hidden=10, max_hidden=60),
             tag="_late")
    gen_gae()
    gen_model()
    gen_ppo()
    gen_ppo_full()


if __name__ == "__main__":
    main()

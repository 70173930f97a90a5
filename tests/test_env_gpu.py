"""GPU parity of the HIP board step against the golden fixtures (captured from
the reference) and against the pinned CPU oracle, through the C ABI."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import golden, golden_files
import oracle as O

pytestmark = pytest.mark.gpu


def _vec(H, W, K, N, seed=0, **kw):
    from ms_amd import EnvConfig, VecMinesweeper
    return VecMinesweeper(N, EnvConfig(H=H, W=W, mine_count=K), seed=seed, **kw)


def _codes(obs: torch.Tensor) -> np.ndarray:
    return O.codes_from_obs(obs.cpu().numpy())


@pytest.mark.parametrize("name", golden_files("traj_*.npz"))
def test_trajectory_golden_gpu(gpu, name):
    """Reference trajectories replayed bit-exact, incl. late-start resets (traj_*_late:
    VecMinesweeper(late_start_cfg, late_start_seed=seed+1) as train_rl.py:350-361)."""
    z = golden(name)
    H, W, K, N, T = (int(z[k]) for k in ("H", "W", "K", "N", "T"))
    late = None
    if "late_prob" in z.files:
        late = dict(prob=float(z["late_prob"]), min_hidden=int(z["late_min"]), max_hidden=int(z["late_max"]))
    v = _vec(H, W, K, N, seed=int(z["seed"]), late_start_cfg=late,
             late_start_seed=int(z["seed"]) + 1 if late else None)
    d = v.reset()
    assert np.array_equal(_codes(d["obs"]), z["reset_codes"])
    mode = int(z["mode"])
    for t in range(T):
        a = v.tape_actions(t, mode)
        assert np.array_equal(a.cpu().numpy(), z["actions"][t]), t
        batch, r, dn, info = v.step(a)
        assert np.array_equal(r.cpu().numpy(), z["rewards"][t]), t
        assert np.array_equal(dn.cpu().numpy(), z["dones"][t]), t
        tens = info.tensors
        assert np.array_equal(tens["outcome"].cpu().numpy(), z["outcome"][t]), t
        assert np.array_equal(tens["step"].cpu().numpy(), z["step"][t]), t
        assert np.array_equal(tens["last_new_reveals"].cpu().numpy(), z["last_new"][t]), t
        assert np.array_equal(tens["revealed_frac"].cpu().numpy(), z["frac"][t]), t
        assert np.array_equal(_codes(batch["obs"]), z["codes"][t]), t
        assert np.array_equal(batch["action_mask"].cpu().numpy(), z["codes"][t] == 0), t
        mines = v.snapshot_tensors()["mine"].cpu().numpy().reshape(N, -1)
        assert np.array_equal(np.packbits(mines, axis=1), z["mines"][t]), t
    assert np.array_equal(v.rng_state(), z["end_states"])
    if late:
        assert np.array_equal(v.late_rng_state(), z["late_state"])


def _diff_run(H, W, K, N, T, mode, seed=0, check_every=1, labels=True, late=None, dbg=0):
    v = _vec(H, W, K, N, seed=seed, late_start_cfg=late, late_start_seed=seed + 1 if late else None)
    if dbg:
        v.set_debug_flags(dbg)
    o = O.OracleVec(H, W, K, N, seed=seed, late_start=late, late_seed=seed + 1 if late else None)
    d = v.reset()
    oo, om = o.reset()
    assert np.array_equal(d["obs"].cpu().numpy(), oo)
    for t in range(T):
        a = v.tape_actions(t, mode)
        a_np = a.cpu().numpy()
        assert np.array_equal(a_np, o.tape(t, mode)), t
        if labels and t % 7 == 3:
            lab, val = v.mine_labels()
            olab, oval = o.labels()
            assert np.array_equal(lab.cpu().numpy(), olab) and np.array_equal(val.cpu().numpy(), oval)
        batch, r, dn, info = v.step(a)
        ref = o.step(a_np)
        tens = info.tensors
        assert np.array_equal(r.cpu().numpy(), ref["reward"]), t
        assert np.array_equal(dn.cpu().numpy(), ref["done"]), t
        assert np.array_equal(tens["outcome"].cpu().numpy(), ref["outcome"]), t
        assert np.array_equal(tens["last_new_reveals"].cpu().numpy(), ref["last_new"]), t
        assert np.array_equal(tens["revealed_frac"].cpu().numpy(), ref["frac"]), t
        if t % check_every == 0:
            assert np.array_equal(batch["obs"].cpu().numpy(), ref["obs"]), t
            assert np.array_equal(batch["action_mask"].cpu().numpy(), ref["mask"]), t
    snap = v.snapshot_tensors()
    osnap = o.snapshot()
    assert np.array_equal(snap["counts"].cpu().numpy().reshape(N, -1), osnap["counts"])
    assert np.array_equal(snap["mine"].cpu().numpy().reshape(N, -1), osnap["mine"])
    assert np.array_equal(snap["step_count"].cpu().numpy(), osnap["step_count"])
    assert np.array_equal(v.rng_state(), o.rng_state())


@pytest.mark.parametrize("H,W,K,N", [(16, 16, 40, 96), (9, 9, 10, 200), (30, 16, 99, 40), (7, 11, 20, 64)])
def test_late_start_matches_oracle(gpu, H, W, K, N):
    """Late-start resets (env.py:416-466) on the HIP path vs the C oracle: the shared
    generator's env-order chain, retries, fallback resets, step counts."""
    late = dict(prob=0.6, min_hidden=3, max_hidden=2 * K, max_attempts=2)
    _diff_run(H, W, K, N, T=60, mode=1, seed=5, check_every=3, labels=False, late=late)


@pytest.mark.parametrize("H,W,K,N", [(16, 16, 40, 256), (9, 9, 10, 300), (30, 16, 99, 64), (7, 11, 20, 64)])
def test_late_start_keyed_matches_oracle(gpu, H, W, K, N):
    """MS_LATE_KEYED (one stream per reset, one wave per env, all resets of a step at once)
    vs the oracle's restatement of the same rule (keyed_late_rng): bit-exact."""
    late = dict(prob=0.6, min_hidden=3, max_hidden=2 * K, max_attempts=2, rng="keyed")
    _diff_run(H, W, K, N, T=60, mode=1, seed=5, check_every=3, labels=False, late=late)


def test_late_start_keyed_sharded_equals_unsharded(gpu):
    """Keyed late starts depend on the GLOBAL env index only: two shards of a 512-env list
    step exactly as the unsharded handle (the shared mode cannot: its stream is env-ordered)."""
    from ms_amd import EnvConfig, VecMinesweeper
    late = dict(prob=0.7, min_hidden=3, max_hidden=60, rng="keyed")
    cfg = EnvConfig(H=16, W=16, mine_count=40)
    full = VecMinesweeper(512, cfg, seed=4, late_start_cfg=late, late_start_seed=9)
    parts = [VecMinesweeper(512, cfg, seed=4, late_start_cfg=late, late_start_seed=9, shard=(r, 2)) for r in range(2)]
    obs = [full.reset()["obs"]] + [p.reset()["obs"] for p in parts]
    assert torch.equal(obs[0], torch.cat(obs[1:]))
    for t in range(40):
        a = full.tape_actions(t, 1)
        b_full, r_full, d_full, _ = full.step(a)
        outs = [p.step(p.tape_actions(t, 1)) for p in parts]
        assert torch.equal(b_full["obs"], torch.cat([o[0]["obs"] for o in outs])), t
        assert torch.equal(r_full, torch.cat([o[1] for o in outs])), t
        assert torch.equal(d_full, torch.cat([o[2] for o in outs])), t
    assert np.array_equal(full.rng_state(), np.concatenate([p.rng_state() for p in parts]))


@pytest.mark.parametrize("H,W,K", [(16, 16, 40), (9, 9, 10), (30, 16, 99), (16, 30, 99), (8, 8, 10)])
@pytest.mark.parametrize("mode", [0, 1])
def test_diff_vs_oracle_benchmark_shapes(gpu, H, W, K, mode):
    _diff_run(H, W, K, N=512, T=120, mode=mode, seed=11)


@pytest.mark.parametrize("H,W,K", [(5, 7, 8), (1, 1, 0), (2, 3, 5), (13, 31, 60), (64, 62, 700),
                                   (64, 1, 10), (1, 62, 12), (4, 4, 15), (6, 6, 0)])
def test_diff_vs_oracle_generic_shapes(gpu, H, W, K):
    _diff_run(H, W, K, N=64, T=60, mode=1, seed=5)


def test_guarantee_off_and_custom_rewards(gpu):
    from ms_amd import EnvConfig, VecMinesweeper
    cfg = EnvConfig(H=8, W=8, mine_count=20, guarantee_safe_neighborhood=False, win_reward=2.5,
                    loss_reward=-0.75, step_penalty=0.01)
    v = VecMinesweeper(128, cfg, seed=2)
    o = O.OracleVec(8, 8, 20, 128, seed=2, guarantee=False, win_reward=2.5, loss_reward=-0.75,
                    step_penalty=0.01)
    v.reset()
    o.reset()
    for t in range(80):
        a = v.tape_actions(t, 1)
        _, r, dn, _ = v.step(a)
        ref = o.step(a.cpu().numpy())
        assert np.array_equal(r.cpu().numpy(), ref["reward"])
        assert np.array_equal(dn.cpu().numpy(), ref["done"])


def test_int32_and_wrapped_actions(gpu):
    v1, v2 = _vec(16, 16, 40, 256, seed=3), _vec(16, 16, 40, 256, seed=3)
    v1.reset()
    v2.reset()
    g = torch.Generator().manual_seed(0)
    for t in range(30):
        a = torch.randint(-10_000, 10_000, (256,), generator=g)
        b1, r1, d1, _ = v1.step(a.to(torch.int32).cuda())
        b2, r2, d2, _ = v2.step(torch.remainder(a, 256).cuda())
        assert torch.equal(b1["obs"], b2["obs"]) and torch.equal(r1, r2) and torch.equal(d1, d2)


def test_bad_action_shape_asserts(gpu):
    v = _vec(8, 8, 10, 4)
    v.reset()
    with pytest.raises(AssertionError):
        v.step(np.zeros(5, np.int64))


def test_sharded_equals_unsharded(gpu):
    from ms_amd import EnvConfig, VecMinesweeper
    cfg = EnvConfig(H=16, W=16, mine_count=40)
    full = VecMinesweeper(1024, cfg, seed=7)
    parts = [VecMinesweeper(1024, cfg, seed=7, shard=(r, 4)) for r in range(4)]
    full.reset()
    for p in parts:
        p.reset()
    for t in range(40):
        a = full.tape_actions(t, 0)
        pa = [p.tape_actions(t, 0) for p in parts]
        assert torch.equal(a, torch.cat(pa))
        bf, rf, _, _ = full.step(a)
        outs = [p.step(x) for p, x in zip(parts, pa)]
        assert torch.equal(bf["obs"], torch.cat([o[0]["obs"] for o in outs]))
        assert torch.equal(rf, torch.cat([o[1] for o in outs]))


def test_full_size_properties(gpu):
    """BASELINE config C2 (16x16x40, N=4096): size-independent invariants."""
    N, H, W, K = 4096, 16, 16, 40
    v = _vec(H, W, K, N, seed=0)
    d = v.reset()
    assert torch.count_nonzero(d["obs"]) == 0 and bool(d["action_mask"].all())
    for t in range(200):
        a = v.tape_actions(t, 1)
        batch, r, dn, info = v.step(a)
        obs, mask = batch["obs"], batch["action_mask"]
        # one-hot: each revealed cell has exactly one count plane; hidden none
        rev = obs[:, 0] > 0
        assert torch.equal(obs[:, 1:].sum(1), rev.float())
        assert torch.equal(mask.view(N, H, W), ~rev)
        # done envs come back fresh
        assert torch.count_nonzero(obs[dn]) == 0
        # rewards take only the three reference values
        vals = torch.unique(r).cpu().numpy()
        allowed = {np.float32(-1e-4), np.float32(-1.0 - 1e-4), np.float32(1.0 - 1e-4)}
        assert set(vals.tolist()) <= {float(x) for x in allowed}
    snap = v.snapshot_tensors()
    fc = snap["first_click"]
    assert torch.equal(snap["mine"][fc].sum((1, 2)), torch.full((int(fc.sum()),), K, device=gpu,
                                                                dtype=torch.int64))
    assert not bool(snap["mine"][~fc].any())


def test_numpy_compat_mode(gpu):
    v = _vec(9, 9, 10, 16, as_numpy=True)
    d = v.reset()
    assert isinstance(d["obs"], np.ndarray) and d["obs"].dtype == np.float32
    assert d["action_mask"].dtype == bool and d["action_mask"].shape == (16, 81)
    b, r, dn, info = v.step(np.zeros(16, np.int32))
    assert r.dtype == np.float32 and dn.dtype == bool
    assert len(info["aux"]) == 16 and set(info["aux"][0]) == {"step", "last_new_reveals", "revealed_frac"}
    assert all(o is None or o in ("win", "loss") for o in info["outcome"])
    e = v.envs[3]
    assert e.first_click_done and e.revealed.shape == (9, 9) and e.mine_mask.sum() == 10
    assert (e.adjacent_counts <= 8).all() and not e.flags.any()


@pytest.mark.parametrize("H,W,K", [(16, 16, 40), (30, 16, 99), (64, 62, 2000), (9, 9, 10), (4, 4, 15)])
def test_parallel_and_serial_placement_agree(gpu, H, W, K):
    """The lane-parallel PCG/Floyd placement and the serial reference-order
    path (its fallback, forced here) give identical boards and RNG states."""
    from ms_amd import _lib as L
    a, b = _vec(H, W, K, 256, seed=21), _vec(H, W, K, 256, seed=21)
    b.set_debug_flags(L.MS_DBG_FORCE_SERIAL_PLACEMENT)
    a.reset()
    b.reset()
    for t in range(40):
        act = a.tape_actions(t, 0)
        ba, ra, da, _ = a.step(act)
        bb, rb, db, _ = b.step(act)
        assert torch.equal(ba["obs"], bb["obs"]) and torch.equal(ra, rb) and torch.equal(da, db), t
        assert np.array_equal(a.rng_state(), b.rng_state()), t


@pytest.mark.parametrize("H,W,K", [(16, 16, 40), (30, 16, 99), (16, 30, 128), (9, 9, 10), (4, 4, 15),
                                   (12, 12, 129), (3, 3, 8)])
def test_fixpoint_chain_and_serial_placement_agree(gpu, H, W, K):
    """All three placement paths (lane-parallel fixpoint K<=128, jump-ahead +
    serial Floyd chain, fully serial reference order) agree with the oracle."""
    from ms_amd import _lib as L
    vs = [_vec(H, W, K, 192, seed=33) for _ in range(3)]
    vs[1].set_debug_flags(2)  # MS_DBG_FORCE_CHAIN_PLACEMENT
    vs[2].set_debug_flags(L.MS_DBG_FORCE_SERIAL_PLACEMENT)
    o = O.OracleVec(H, W, K, 192, seed=33)
    o.reset()
    for v in vs:
        v.reset()
    for t in range(30):
        act = vs[0].tape_actions(t, 0)
        ref = o.step(act.cpu().numpy())
        for v in vs:
            b, r, d, _ = v.step(act)
            assert np.array_equal(b["obs"].cpu().numpy(), ref["obs"]), t
            assert np.array_equal(r.cpu().numpy(), ref["reward"]), t
        st = o.rng_state()
        for v in vs:
            assert np.array_equal(v.rng_state(), st), t


@pytest.mark.parametrize("H,W,K,N", [(9, 9, 10, 203), (8, 8, 10, 130), (9, 9, 16, 64), (9, 9, 1, 33),
                                     (9, 9, 10, 1), (9, 9, 10, 6)])
@pytest.mark.parametrize("mode", [0, 1])
def test_packed_step_equals_one_board_per_wave(gpu, H, W, K, N, mode):
    """k_step_packed (four boards per wave in 16-lane DPP rows, per-board RNG in VGPRs,
    register Floyd chain) is bit-exact with k_step (one board per wave): every output, the
    mines and the RNG state, at env counts that leave a partial last wave; K = 16 and K = 1
    are the packed placement's edges. Its forced serial fallback and the two-boards-per-wave
    form (32-lane groups) agree as well."""
    from ms_amd import _lib as L
    a, b, c, d = (_vec(H, W, K, N, seed=17) for _ in range(4))
    b.set_debug_flags(L.MS_DBG_ONE_BOARD_PER_WAVE)
    c.set_debug_flags(L.MS_DBG_FORCE_SERIAL_PLACEMENT)
    d.set_debug_flags(L.MS_DBG_TWO_BOARDS_PER_WAVE)
    for v in (a, b, c, d):
        v.reset()
    for t in range(80):
        act = a.tape_actions(t, mode)
        outs = [v.step(act) for v in (a, b, c, d)]
        for o in outs[1:]:
            assert torch.equal(outs[0][0]["obs"], o[0]["obs"]), t
            assert torch.equal(outs[0][0]["action_mask"], o[0]["action_mask"]), t
            assert torch.equal(outs[0][1], o[1]) and torch.equal(outs[0][2], o[2]), t
            for k, x in outs[0][3].tensors.items():
                assert torch.equal(x, o[3].tensors[k]), (t, k)
        st = a.rng_state()
        assert all(np.array_equal(st, v.rng_state()) for v in (b, c, d)), t
    sa, sb = a.snapshot_tensors(), b.snapshot_tensors()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


@pytest.mark.parametrize("K,N", [(40, 203), (40, 4), (40, 1), (48, 66), (1, 37), (10, 64), (47, 130)])
@pytest.mark.parametrize("mode", [0, 1])
def test_packed16_step_equals_one_board_per_wave(gpu, K, N, mode):
    """16x16 boards four to a wave (k_step_packed with place_packed3 and pk_emit16; forced below
    its env-count threshold) are bit-exact with k_step: every output, the boards and the RNG
    state, including the serial placement fallback; K = 48 / 47 fill the three Floyd slots per
    lane, K = 1 the first; N = 203 / 130 / 37 leave a partial last wave."""
    from ms_amd import _lib as L
    a, b, c = (_vec(16, 16, K, N, seed=23) for _ in range(3))
    a.set_debug_flags(L.MS_DBG_FORCE_PACKED)
    b.set_debug_flags(L.MS_DBG_ONE_BOARD_PER_WAVE)
    c.set_debug_flags(L.MS_DBG_FORCE_PACKED | L.MS_DBG_FORCE_SERIAL_PLACEMENT)
    for v in (a, b, c):
        v.reset()
    for t in range(60):
        act = a.tape_actions(t, mode)
        outs = [v.step(act) for v in (a, b, c)]
        for o in outs[1:]:
            assert torch.equal(outs[0][0]["obs"], o[0]["obs"]), t
            assert torch.equal(outs[0][0]["action_mask"], o[0]["action_mask"]), t
            assert torch.equal(outs[0][1], o[1]) and torch.equal(outs[0][2], o[2]), t
            for k, x in outs[0][3].tensors.items():
                assert torch.equal(x, o[3].tensors[k]), (t, k)
        st = a.rng_state()
        assert all(np.array_equal(st, v.rng_state()) for v in (b, c)), t
    sa, sb = a.snapshot_tensors(), b.snapshot_tensors()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


@pytest.mark.parametrize("N", [203, 512])
@pytest.mark.parametrize("mode", [0, 1])
def test_packed16_step_vs_oracle(gpu, N, mode):
    """The 16x16 four-boards-a-wave step (k_step_packed, forced below its env-count threshold)
    directly against the C oracle, not only against k_step: obs, mask, rewards, dones, outcome,
    labels, counts, mines and RNG state over 120 steps (N = 203 leaves a partial last wave)."""
    from ms_amd import _lib as L
    _diff_run(16, 16, 40, N=N, T=120, mode=mode, seed=13, dbg=L.MS_DBG_FORCE_PACKED)


def test_packed16_default_dispatch_at_65536(gpu):
    """At 65,536 16x16x40 envs the dispatcher takes the packed kernel by itself (no flag); it
    stays bit-exact with the one-board kernel over 25 steps (N = 65,538 leaves a partial wave)."""
    from ms_amd import _lib as L
    N = 65538
    a, b = _vec(16, 16, 40, N, seed=5), _vec(16, 16, 40, N, seed=5)
    b.set_debug_flags(L.MS_DBG_ONE_BOARD_PER_WAVE)
    a.reset()
    b.reset()
    for t in range(25):
        act = a.tape_actions(t, 0)
        (ba, ra, da, ia), (bb, rb, db, ib) = a.step(act), b.step(act)
        assert torch.equal(ba["obs"], bb["obs"]) and torch.equal(ba["action_mask"], bb["action_mask"]), t
        assert torch.equal(ra, rb) and torch.equal(da, db), t
        for k, x in ia.tensors.items():
            assert torch.equal(x, ib.tensors[k]), (t, k)
    assert np.array_equal(a.rng_state(), b.rng_state())


def test_packed_step_misaligned_obs_falls_back(gpu):
    """An obs base that is not 16-B aligned (a view one float in) takes k_step; results equal."""
    from ms_amd import _lib as L
    a, b = _vec(9, 9, 10, 40, seed=3), _vec(9, 9, 10, 40, seed=3)
    b.set_debug_flags(L.MS_DBG_ONE_BOARD_PER_WAVE)
    a.reset()
    b.reset()
    for t in range(10):
        act = a.tape_actions(t, 1)
        big = torch.empty(40 * 810 + 1, device="cuda")
        obs = big[1:].view(40, 10, 9, 9)
        out = dict(obs=obs, action_mask=torch.empty(40, 81, dtype=torch.bool, device="cuda"),
                   rewards=torch.empty(40, device="cuda"), dones=torch.empty(40, dtype=torch.bool, device="cuda"))
        a.step(act, out=out)
        mask = out["action_mask"]
        ba, ra, da, _ = b.step(act)
        assert torch.equal(out["rewards"], ra) and torch.equal(out["dones"], da), t
        assert torch.equal(obs, ba["obs"]) and torch.equal(mask, ba["action_mask"]), t


_RUN_KEYS = ("actions", "obs", "action_mask", "rewards", "dones", "step", "last_new_reveals", "revealed_frac",
             "outcome")


@pytest.mark.parametrize("H,W,K", [(16, 16, 40), (9, 9, 10), (30, 16, 99), (16, 30, 99), (8, 8, 10), (5, 7, 8)])
@pytest.mark.parametrize("mode", [0, 1])
def test_run_tape_equals_step_loop(gpu, H, W, K, mode):
    """ms_run_tape (T tape steps in one launch, boards held in registers) is bit-exact with
    T x (ms_tape_actions + ms_step); a second launch continues identically."""
    N, T = 300, 40
    a, b = _vec(H, W, K, N, seed=9), _vec(H, W, K, N, seed=9)
    a.reset()
    b.reset()
    ref = {k: [] for k in _RUN_KEYS}
    for t in range(2 * T):
        act = a.tape_actions(7 + t, mode)
        batch, r, d, info = a.step(act)
        vals = dict(actions=act, obs=batch["obs"], action_mask=batch["action_mask"], rewards=r, dones=d,
                    **{k: v for k, v in info.tensors.items() if k != "done"})
        for k in _RUN_KEYS:
            ref[k].append(vals[k].clone())
    o1 = b.run_tape(7, T, mode, slots=True)
    o2 = b.run_tape(7 + T, T, mode, slots=False)
    for k in _RUN_KEYS:
        assert torch.equal(torch.stack(ref[k][:T]), o1[k]), k
        assert torch.equal(ref[k][-1], o2[k]), k
    assert np.array_equal(a.rng_state(), b.rng_state())
    sa, sb = a.snapshot_tensors(), b.snapshot_tensors()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


@pytest.mark.parametrize("H,W,K,N,slots", [(9, 9, 10, 300, True), (9, 9, 10, 203, False), (8, 8, 10, 130, True),
                                           (9, 9, 16, 64, True)])
@pytest.mark.parametrize("mode", [0, 1])
def test_run_tape_packed_equals_one_board_per_wave(gpu, H, W, K, N, slots, mode):
    """k_run_packed (four boards per wave; two with MS_DBG_TWO_BOARDS_PER_WAVE) is bit-exact
    with k_run (one board per wave) over two launches: every output slot, the boards and the
    RNG state; N = 203 / 130 leave a partial last wave."""
    from ms_amd import _lib as L
    vs = [_vec(H, W, K, N, seed=13) for _ in range(3)]
    vs[1].set_debug_flags(L.MS_DBG_ONE_BOARD_PER_WAVE)
    vs[2].set_debug_flags(L.MS_DBG_TWO_BOARDS_PER_WAVE)
    for v in vs:
        v.reset()
    for t0 in (5, 40):
        outs = [v.run_tape(t0, 35, mode, slots=slots) for v in vs]
        for o in outs[1:]:
            for k in _RUN_KEYS:
                assert torch.equal(outs[0][k], o[k]), (t0, k)
    st = vs[0].rng_state()
    assert all(np.array_equal(st, v.rng_state()) for v in vs[1:])
    snaps = [v.snapshot_tensors() for v in vs]
    for sn in snaps[1:]:
        for k in snaps[0]:
            assert torch.equal(snaps[0][k], sn[k]), k


@pytest.mark.parametrize("K,N,slots", [(40, 203, True), (40, 130, False), (48, 66, True)])
@pytest.mark.parametrize("mode", [0, 1])
def test_run_tape_packed16_equals_one_board_per_wave(gpu, K, N, slots, mode):
    """16x16 k_run_packed (four boards per wave, place_packed3, pk_emit16; forced below its env-count
    threshold) is bit-exact with k_run over two launches: every output slot, boards and RNG state."""
    from ms_amd import _lib as L
    vs = [_vec(16, 16, K, N, seed=29) for _ in range(2)]
    vs[0].set_debug_flags(L.MS_DBG_FORCE_PACKED)
    vs[1].set_debug_flags(L.MS_DBG_ONE_BOARD_PER_WAVE)
    for v in vs:
        v.reset()
    for t0 in (3, 40):
        outs = [v.run_tape(t0, 30, mode, slots=slots) for v in vs]
        for k in _RUN_KEYS:
            assert torch.equal(outs[0][k], outs[1][k]), (t0, k)
    assert np.array_equal(vs[0].rng_state(), vs[1].rng_state())
    sa, sb = vs[0].snapshot_tensors(), vs[1].snapshot_tensors()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


def test_run_tape_sharded_and_late_start(gpu):
    from ms_amd import EnvConfig, VecMinesweeper
    from ms_amd._lib import MsEnvError
    cfg = EnvConfig(H=16, W=16, mine_count=40)
    full = VecMinesweeper(512, cfg, seed=4)
    parts = [VecMinesweeper(512, cfg, seed=4, shard=(r, 2)) for r in range(2)]
    full.reset()
    for p in parts:
        p.reset()
    of = full.run_tape(3, 25, 1, slots=False)
    op = [p.run_tape(3, 25, 1, slots=False) for p in parts]
    for k in _RUN_KEYS:
        assert torch.equal(of[k], torch.cat([o[k] for o in op])), k
    late = _vec(9, 9, 10, 8, late_start_cfg=dict(prob=0.5, min_hidden=3, max_hidden=20), late_start_seed=1)
    late.reset()
    with pytest.raises(MsEnvError):
        late.run_tape(0, 4, 0)


@pytest.mark.parametrize("H,W,K,N", [(16, 16, 40, 4096), (9, 9, 10, 8192), (30, 16, 99, 8192), (16, 30, 99, 8192)],
                         ids=["C2", "C3", "C5", "C5-transposed"])
def test_full_size_configs_vs_oracle(gpu, H, W, K, N):
    """BASELINE configs at their full env counts (C3 9x9x10 and C5 30x16x99 at N=8192 -- C5's
    8 GPUs x 1024 envs is the same global env list), 20 steps of each tape: obs, mask, rewards,
    dones, outcome, aux, labels, counts, mines and RNG state bit-exact with the C oracle."""
    _diff_run(H, W, K, N=N, T=20, mode=0, seed=0, check_every=1)
    _diff_run(H, W, K, N=N, T=20, mode=1, seed=1, check_every=4)


def test_c4_eight_shards_equal_unsharded_32768(gpu):
    """BASELINE C4 (16x16x40, N=32768 over 8 GPUs at 4096 each): the 8 shards of the global
    env list, stepped side by side in one process, equal one unsharded 32768-env handle bit
    for bit (obs, mask, rewards, dones, aux, RNG state), so the 8-GPU run is trajectory-
    identical to a single device."""
    from ms_amd import EnvConfig, VecMinesweeper
    cfg = EnvConfig(H=16, W=16, mine_count=40)
    N = 32768
    full = VecMinesweeper(N, cfg, seed=0)
    parts = [VecMinesweeper(N, cfg, seed=0, shard=(r, 8)) for r in range(8)]
    assert all(p.num_envs == 4096 for p in parts)
    full.reset()
    for p in parts:
        p.reset()
    for t in range(20):
        a = full.tape_actions(t, 1)
        pa = [p.tape_actions(t, 1) for p in parts]
        assert torch.equal(a, torch.cat(pa)), t
        bf, rf, df, inf = full.step(a)
        outs = [p.step(x) for p, x in zip(parts, pa)]
        assert torch.equal(bf["obs"], torch.cat([o[0]["obs"] for o in outs])), t
        assert torch.equal(bf["action_mask"], torch.cat([o[0]["action_mask"] for o in outs])), t
        assert torch.equal(rf, torch.cat([o[1] for o in outs])), t
        assert torch.equal(df, torch.cat([o[2] for o in outs])), t
        for k in ("outcome", "step", "last_new_reveals", "revealed_frac"):
            assert torch.equal(inf.tensors[k], torch.cat([o[3].tensors[k] for o in outs])), (t, k)
    assert np.array_equal(full.rng_state(), np.concatenate([p.rng_state() for p in parts]))

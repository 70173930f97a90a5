"""Pin the CPU oracle (oracle/ms_oracle.c) before trusting it as the checker.

Against numpy itself (the third-party arithmetic, env.py:49/309/393-394) and
against the golden fixtures captured from the reference (tests/golden/).
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import golden, golden_files
import oracle as O

M64 = (1 << 64) - 1


def np_state(g):
    s = g.bit_generator.state
    st, inc = s["state"]["state"], s["state"]["inc"]
    return np.array([st >> 64, st & M64, inc >> 64, inc & M64, s["has_uint32"], s["uinteger"]],
                    dtype=np.uint64)


@pytest.mark.parametrize("seed", [0, 1, 7, 12345, 2**31 - 2, 2**32, 2**40 + 5, 2**63 + 11])
def test_seed_sequence_pcg64_matches_numpy(seed):
    assert np.array_equal(O.seed_state(seed), np_state(np.random.default_rng(seed)))


@pytest.mark.parametrize("j", [1, 2, 7, 246, 4095, 2**31 - 2, 2**32 - 2])
def test_bounded_draws_match_numpy(j):
    g = np.random.default_rng(99)
    g.integers(0, 5)  # leave a buffered half-word behind
    st = np_state(g)
    out, st2 = O.bounded_draws(st, j, 500)
    ref = g.integers(0, j + 1, size=500, dtype=np.int64)
    assert np.array_equal(out.astype(np.int64), ref)
    assert np.array_equal(st2, np_state(g))


def test_u64_and_random_match_numpy():
    g = np.random.default_rng(5)
    st = np_state(g)
    out, _ = O.u64_draws(st, 100)
    ref = g.bit_generator.random_raw(100)
    assert np.array_equal(out, ref.astype(np.uint64))


@pytest.mark.parametrize("pop,k", [(247, 40), (72, 10), (471, 99), (15, 15), (3968, 700), (9, 1)])
def test_choice_noreplace_matches_numpy(pop, k):
    for seed in range(5):
        g = np.random.default_rng(seed)
        st = np_state(g)
        out, st2 = O.choice_noreplace(st, pop, k)
        ref = g.choice(pop, size=k, replace=False)
        assert np.array_equal(out, ref)
        assert np.array_equal(st2, np_state(g))


@pytest.mark.parametrize("name", golden_files("seeds_*.npz"))
def test_env_seed_derivation_golden(name):
    z = golden(name)
    seeds, st = O.env_seeds(int(z["base"]), len(z["seeds"]))
    assert np.array_equal(seeds, z["seeds"])
    assert np.array_equal(st, z["base_state_after"])
    for i, s in enumerate(seeds):
        assert np.array_equal(O.seed_state(int(s)), z["env_states"][i])


@pytest.mark.parametrize("name", golden_files("place_*.npz"))
def test_mine_placement_golden(name):
    z = golden(name)
    H, W, K, g = int(z["H"]), int(z["W"]), int(z["K"]), bool(z["guarantee"])
    for i in range(len(z["seeds"])):
        r, c = z["clicks"][i]
        mine, cnt, st = O.place_probe(H, W, K, g, int(z["seeds"][i]), int(r), int(c))
        assert np.array_equal(mine, z["mines"][i]), (name, i)
        assert np.array_equal(cnt, z["counts"][i]), (name, i)
        assert np.array_equal(st, z["states"][i]), (name, i)


def replay_traj(z, nthreads=1):
    H, W, K, N, T = (int(z[k]) for k in ("H", "W", "K", "N", "T"))
    late = None
    if "late_prob" in z.files:
        late = dict(prob=float(z["late_prob"]), min_hidden=int(z["late_min"]),
                    max_hidden=int(z["late_max"]))
    v = O.OracleVec(H, W, K, N, seed=int(z["seed"]), late_start=late)
    obs, mask = v.reset()
    assert np.array_equal(O.codes_from_obs(obs), z["reset_codes"])
    mode = int(z["mode"])
    for t in range(T):
        a = v.tape(t, mode)
        assert np.array_equal(a, z["actions"][t]), t
        out = v.step(a, nthreads=nthreads)
        assert np.array_equal(out["reward"], z["rewards"][t]), t
        assert np.array_equal(out["done"], z["dones"][t]), t
        assert np.array_equal(out["outcome"], z["outcome"][t]), t
        assert np.array_equal(out["step"], z["step"][t]), t
        assert np.array_equal(out["last_new"], z["last_new"][t]), t
        assert np.array_equal(out["frac"], z["frac"][t]), t
        assert np.array_equal(O.codes_from_obs(out["obs"]), z["codes"][t]), t
        assert np.array_equal(out["mask"], z["codes"][t] == 0), t
        snap = v.snapshot()
        assert np.array_equal(np.packbits(snap["mine"], axis=1), z["mines"][t]), t
    assert np.array_equal(v.rng_state(), z["end_states"])


@pytest.mark.parametrize("name", golden_files("traj_*.npz"))
def test_trajectory_golden(name):
    replay_traj(golden(name))


def test_trajectory_threaded_equals_serial():
    z = golden("traj_16x16x40_m1.npz")
    replay_traj(z, nthreads=4)


def test_sharded_oracle_equals_unsharded():
    full = O.OracleVec(9, 9, 10, 64, seed=3)
    parts = [O.OracleVec(9, 9, 10, 64, seed=3, env_begin=b, env_count=16) for b in (0, 16, 32, 48)]
    full.reset()
    for p in parts:
        p.reset()
    for t in range(50):
        a = full.tape(t, 0)
        assert np.array_equal(a, np.concatenate([p.tape(t, 0) for p in parts]))
        o = full.step(a)
        po = [p.step(a[16 * i:16 * (i + 1)]) for i, p in enumerate(parts)]
        assert np.array_equal(o["obs"], np.concatenate([x["obs"] for x in po]))
        assert np.array_equal(o["reward"], np.concatenate([x["reward"] for x in po]))


def test_gae_golden_bitexact():
    z = golden("gae.npz")
    T, N = int(z["T"]), int(z["N"])
    adv, ret = O.gae(z["rewards"].reshape(T, N), z["values"].reshape(T, N),
                     z["dones"].reshape(T, N), z["last_values"], float(z["gamma"]), float(z["lam"]))
    assert np.array_equal(adv.reshape(-1), z["advantages"])
    assert np.array_equal(ret.reshape(-1), z["returns"])


def test_negative_and_large_actions_wrap_python_style():
    v = O.OracleVec(8, 8, 10, 4, seed=0)
    w = O.OracleVec(8, 8, 10, 4, seed=0)
    v.reset(); w.reset()
    a = np.array([-1, 64 + 5, -65, 3], np.int64)
    o1 = v.step(a)
    o2 = w.step(np.mod(a, 64))
    for k in ("reward", "done", "step", "last_new", "frac"):
        assert np.array_equal(o1[k], o2[k])
    assert np.array_equal(o1["obs"], o2["obs"])


def test_cpu_baseline_runner_equals_step_loop():
    """mso_run_baseline (bench.py's cpu_baseline: per-thread env blocks, no per-step sync) is
    the same computation as T x (tape + step) over the batch."""
    import oracle as O
    H, W, K, N, T = 9, 9, 10, 96, 25
    a, b = O.OracleVec(H, W, K, N, seed=4), O.OracleVec(H, W, K, N, seed=4)
    a.reset()
    b.reset()
    for t in range(T):
        a.step(a.tape(t, 1))
    bufs = (np.zeros((N, 10, H, W), np.float32), np.zeros((N, H * W), np.uint8), np.zeros(N, np.float32),
            np.zeros(N, np.uint8), np.zeros(N, np.int32), np.zeros(N, np.int32), np.zeros(N, np.float64),
            np.zeros(N, np.int8))
    b.run_baseline(0, T, 1, 5, bufs)
    assert np.array_equal(a.rng_state(), b.rng_state())
    sa, sb = a.snapshot(), b.snapshot()
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k


def _late_run(late, n=64, begin=0, count=None, T=40, nthreads=1):
    v = O.OracleVec(16, 16, 40, n, seed=3, env_begin=begin, env_count=count, late_start=late, late_seed=7)
    out = [v.reset()[0]]
    for t in range(T):
        a = v.tape(t, 1)
        out.append(v.step(a, nthreads=nthreads)["obs"])
    return np.stack(out), v.rng_state()


def test_keyed_late_start_sharded_and_threaded_equal_unsharded():
    """MS_LATE_KEYED restated in the oracle: a reset's stream depends on (seed, GLOBAL env, the
    env's own generator state) only, so shards and threads reproduce the unsharded serial run."""
    late = dict(prob=0.7, min_hidden=3, max_hidden=60, rng="keyed")
    full, st = _late_run(late)
    parts = [_late_run(late, begin=b, count=32) for b in (0, 32)]
    assert np.array_equal(full, np.concatenate([p[0] for p in parts], axis=1))
    assert np.array_equal(st, np.concatenate([p[1] for p in parts]))
    thr, st_thr = _late_run(late, nthreads=4)
    assert np.array_equal(full, thr) and np.array_equal(st, st_thr)
    shared, _ = _late_run(dict(late, rng="shared"))
    assert not np.array_equal(full, shared)  # a different stream of draws


def test_keyed_late_start_same_distribution_as_shared():
    """Same procedure (env.py:416-466), different draws: over 2,000 resets the fraction of
    late-started boards and the mean number of revealed cells agree with the shared generator."""
    stats = {}
    for mode in ("shared", "keyed"):
        v = O.OracleVec(16, 16, 40, 2000, seed=1, late_start=dict(prob=0.5, min_hidden=5, max_hidden=80, rng=mode),
                        late_seed=11)
        v.reset()
        snap = v.snapshot()
        started = snap["first_click"].astype(bool)
        rev = snap["revealed"].reshape(2000, -1).sum(1)
        stats[mode] = (started.mean(), rev[started].mean(), (256 - 40 - rev[started]).max())
    (f_s, r_s, h_s), (f_k, r_k, h_k) = stats["shared"], stats["keyed"]
    assert abs(f_s - 0.5) < 0.05 and abs(f_k - 0.5) < 0.05, (f_s, f_k)
    assert abs(r_s - r_k) < 0.05 * r_s, (r_s, r_k)
    assert h_s <= 80 and h_k <= 80  # every late-started board ends within max_hidden safe cells

"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU restatement (ms_oracle.c).

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg. The product package (minesweeper-ppo_amd/ms_amd) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libms_oracle.so")

_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or (
        os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "ms_oracle.c"))
    ):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


class _Cfg(ctypes.Structure):
    _fields_ = [("H", ctypes.c_int32), ("W", ctypes.c_int32), ("mine_count", ctypes.c_int32),
                ("guarantee_safe_neighborhood", ctypes.c_int32), ("win_reward", ctypes.c_double),
                ("loss_reward", ctypes.c_double), ("step_penalty", ctypes.c_double)]


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i64, u64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int32
        L.mso_create.argtypes = [ctypes.POINTER(_Cfg), i64, u64, i64, i64, ctypes.POINTER(vp)]
        L.mso_destroy.argtypes = [vp]
        L.mso_destroy.restype = None
        L.mso_set_late_start.argtypes = [vp, ctypes.c_double, i32, i32, i32, i32, u64]
        L.mso_set_late_start_mode.argtypes = [vp, i32]
        L.mso_reset.argtypes = [vp, vp, vp]
        L.mso_step.argtypes = [vp] + [vp] * 9 + [i32]
        L.mso_step_i32.argtypes = [vp] + [vp] * 9 + [i32]
        L.mso_labels.argtypes = [vp, vp, vp]
        L.mso_snapshot.argtypes = [vp, vp, vp, vp, vp, vp]
        L.mso_rng_state.argtypes = [vp, vp]
        L.mso_tape_actions.argtypes = [vp, u64, i32, vp]
        L.mso_run_baseline.argtypes = [vp, u64, i64, i32, i32] + [vp] * 8
        L.mso_gae.argtypes = [vp, vp, vp, vp, i32, i64, ctypes.c_float, ctypes.c_float, vp, vp]
        L.mso_gae.restype = None
        L.mso_seed_state.argtypes = [u64, vp]
        L.mso_seed_state.restype = None
        L.mso_bounded_draws.argtypes = [vp, u64, i64, vp]
        L.mso_bounded_draws.restype = None
        L.mso_u64_draws.argtypes = [vp, i64, vp]
        L.mso_u64_draws.restype = None
        L.mso_choice_noreplace.argtypes = [vp, i64, i64, vp]
        L.mso_choice_noreplace.restype = None
        L.mso_env_seeds.argtypes = [u64, i64, vp, vp]
        L.mso_env_seeds.restype = None
        L.mso_splitmix64.argtypes = [u64]
        L.mso_splitmix64.restype = u64
        L.mso_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise RuntimeError(lib().mso_last_error().decode())


# late_start_cfg["rng"]: "shared" = the reference's one generator; "keyed" = MS_LATE_KEYED
LATE_MODES = {"shared": 0, "keyed": 1}


class OracleVec:
    """Same state machine as VecMinesweeper, host arrays, one C call per method."""

    def __init__(self, H, W, K, n_total, seed=0, env_begin=0, env_count=None, guarantee=True,
                 win_reward=1.0, loss_reward=-1.0, step_penalty=1e-4, late_start=None,
                 late_seed=None):
        self.H, self.W, self.K = H, W, K
        self.A = H * W
        self.n = n_total - env_begin if env_count is None else env_count
        self.env_begin = env_begin
        cfg = _Cfg(H, W, K, int(guarantee), win_reward, loss_reward, step_penalty)
        h = ctypes.c_void_p()
        _check(lib().mso_create(ctypes.byref(cfg), n_total, seed, env_begin, self.n, ctypes.byref(h)))
        self._h = h
        if late_start:
            ls = dict(late_start)
            mn = int(ls.get("min_hidden", 5))
            lib().mso_set_late_start(h, float(ls.get("prob", 0.0)), mn, int(ls.get("max_hidden", mn)),
                                     int(ls.get("max_attempts", 3)),
                                     int(ls.get("max_extra_steps", H * W)),
                                     int(late_seed if late_seed is not None else seed + 1))
            _check(lib().mso_set_late_start_mode(h, LATE_MODES[ls.get("rng", "shared")]))

    def __del__(self):
        if getattr(self, "_h", None) is not None and _lib is not None:
            _lib.mso_destroy(self._h)
            self._h = None

    def reset(self):
        obs = np.zeros((self.n, 10, self.H, self.W), np.float32)
        mask = np.zeros((self.n, self.A), np.uint8)
        _check(lib().mso_reset(self._h, _p(obs), _p(mask)))
        return obs, mask.astype(bool)

    def step(self, actions, nthreads=1, want_obs=True):
        actions = np.ascontiguousarray(actions)
        n = self.n
        obs = np.zeros((n, 10, self.H, self.W), np.float32) if want_obs else None
        mask = np.zeros((n, self.A), np.uint8) if want_obs else None
        rew = np.zeros(n, np.float32)
        done = np.zeros(n, np.uint8)
        step = np.zeros(n, np.int32)
        lnew = np.zeros(n, np.int32)
        frac = np.zeros(n, np.float64)
        outc = np.zeros(n, np.int8)
        fn = lib().mso_step if actions.dtype == np.int64 else lib().mso_step_i32
        if actions.dtype not in (np.int64, np.int32):
            actions = actions.astype(np.int64)
            fn = lib().mso_step
        _check(fn(self._h, _p(actions), _p(obs), _p(mask), _p(rew), _p(done), _p(step), _p(lnew),
                  _p(frac), _p(outc), nthreads))
        return dict(obs=obs, mask=None if mask is None else mask.astype(bool), reward=rew,
                    done=done.astype(bool), step=step, last_new=lnew, frac=frac, outcome=outc)

    def step_into(self, actions, obs, mask, rew, done, step, lnew, frac, outc, nthreads=1):
        """Zero-allocation step for the CPU-baseline timer (caller-owned buffers)."""
        _check(lib().mso_step(self._h, _p(actions), _p(obs), _p(mask), _p(rew), _p(done), _p(step),
                              _p(lnew), _p(frac), _p(outc), nthreads))

    def labels(self):
        lab = np.zeros((self.n, self.H, self.W), np.float32)
        val = np.zeros((self.n, self.H, self.W), np.uint8)
        _check(lib().mso_labels(self._h, _p(lab), _p(val)))
        return lab, val.astype(bool)

    def snapshot(self):
        mine = np.zeros((self.n, self.A), np.uint8)
        rev = np.zeros((self.n, self.A), np.uint8)
        cnt = np.zeros((self.n, self.A), np.uint8)
        fc = np.zeros(self.n, np.uint8)
        sc = np.zeros(self.n, np.int32)
        _check(lib().mso_snapshot(self._h, _p(mine), _p(rev), _p(cnt), _p(fc), _p(sc)))
        return dict(mine=mine.astype(bool), revealed=rev.astype(bool), counts=cnt,
                    first_click=fc.astype(bool), step_count=sc)

    def rng_state(self):
        out = np.zeros((self.n, 6), np.uint64)
        _check(lib().mso_rng_state(self._h, _p(out)))
        return out

    def run_baseline(self, t0, steps, mode, nthreads, bufs):
        """CPU baseline: ``steps`` x (tape action + board step) for every env on ``nthreads``
        threads that each own a block of envs for the whole run (no per-step sync).
        ``bufs`` = (obs, mask, rew, done, step, lnew, frac, outc) caller arrays."""
        _check(lib().mso_run_baseline(self._h, t0, steps, mode, nthreads, *[_p(b) for b in bufs]))

    def tape(self, t, mode=0, out=None):
        a = np.zeros(self.n, np.int64) if out is None else out
        _check(lib().mso_tape_actions(self._h, t, mode, _p(a)))
        return a


def gae(rewards, values, dones, last_values, gamma=0.995, lam=0.95):
    T, N = rewards.shape
    adv = np.zeros((T, N), np.float32)
    ret = np.zeros((T, N), np.float32)
    lib().mso_gae(_p(np.ascontiguousarray(rewards, np.float32)),
                  _p(np.ascontiguousarray(values, np.float32)),
                  _p(np.ascontiguousarray(dones, np.uint8)),
                  _p(np.ascontiguousarray(last_values, np.float32)), T, N,
                  float(np.float32(gamma)), float(np.float32(gamma * lam)), _p(adv), _p(ret))
    return adv, ret


def seed_state(seed):
    out = np.zeros(6, np.uint64)
    lib().mso_seed_state(seed, _p(out))
    return out


def env_seeds(base_seed, n):
    out = np.zeros(n, np.int64)
    st = np.zeros(6, np.uint64)
    lib().mso_env_seeds(base_seed, n, _p(out), _p(st))
    return out, st


def bounded_draws(state, j, n):
    st = np.array(state, np.uint64)
    out = np.zeros(n, np.uint64)
    lib().mso_bounded_draws(_p(st), j, n, _p(out))
    return out, st


def u64_draws(state, n):
    st = np.array(state, np.uint64)
    out = np.zeros(n, np.uint64)
    lib().mso_u64_draws(_p(st), n, _p(out))
    return out, st


def choice_noreplace(state, pop, k):
    st = np.array(state, np.uint64)
    out = np.zeros(k, np.int64)
    lib().mso_choice_noreplace(_p(st), pop, k, _p(out))
    return out, st


def splitmix64(x):
    return int(lib().mso_splitmix64(x))


def codes_from_obs(obs):
    """[N,10,H,W] one-hot obs -> [N,A] u8 code, same convention as gen_golden.obs_codes."""
    N = obs.shape[0]
    rev = obs[:, 0] > 0
    cnt = np.argmax(obs[:, 1:], axis=1)
    has = obs[:, 1:].sum(axis=1)
    code = np.where(rev, 1 + cnt * (has > 0), 0).astype(np.uint8)
    code = np.where(rev & (has == 0), 255, code).astype(np.uint8)
    return code.reshape(N, -1)


def place_probe(H, W, K, guarantee, seed, r, c):
    L = lib()
    L.mso_place_probe.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_uint64, ctypes.c_int32,
                                  ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    cfg = _Cfg(H, W, K, int(guarantee), 1.0, -1.0, 1e-4)
    mine = np.zeros(H * W, np.uint8)
    cnt = np.zeros(H * W, np.uint8)
    st = np.zeros(6, np.uint64)
    _check(L.mso_place_probe(ctypes.byref(cfg), seed, r, c, _p(mine), _p(cnt), _p(st)))
    return mine.astype(bool), cnt, st

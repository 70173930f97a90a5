"""Device-resident drop-in for the reference's VecMinesweeper.

Reference API (minesweeper/env.py):
  EnvConfig                       env.py:19-30
  VecMinesweeper(num_envs, cfg, seed=0, late_start_cfg=None, late_start_seed=None)
                                  env.py:382-403
  .reset() -> {"obs", "action_mask"}                    env.py:468-477
  .step(actions) -> (batch, rewards, dones, infos)      env.py:479-511
  .action_space(), .obs_channels()                      env.py:513-517
  .num_envs, .cfg, .envs[i]                             (eval.py:350-398, train_rl.py:205-212)

Same method names, shapes, dtypes and error behaviour (AssertionError on a
bad action shape, TypeError on unknown EnvConfig keys). Differences, all
opt-in or additive:
  * arrays are torch tensors on the HIP device (``as_numpy=True`` returns
    numpy copies for unchanged host callers);
  * ``infos`` is a lazy mapping — its lists are built only when indexed;
  * ``shard=(rank, world)`` takes a contiguous block of the GLOBAL env list,
    so a sharded run is trajectory-identical to one device;
  * ``step(..., out=...)`` writes into caller tensors (the rollout buffer's
    next row) instead of allocating.
Every call goes through libmsenv.so (HIP); there is no CPU path.
"""
from __future__ import annotations

from collections.abc import Mapping
from dataclasses import dataclass
from enum import Enum
from typing import Any, Dict, Optional, Tuple

import ctypes
import numpy as np
import torch

from . import _lib as L


class SolverPreset(str, Enum):
    ZF = "zf"


@dataclass
class EnvConfig:
    """Same fields and defaults as env.py:19-30."""
    H: int = 8
    W: int = 8
    mine_count: int = 10
    guarantee_safe_neighborhood: bool = True
    use_pair_constraints: bool | None = None  # deprecated, inert (as in the reference)
    solver_preset: str = SolverPreset.ZF.value

    win_reward: float = 1.0
    loss_reward: float = -1.0
    step_penalty: float = 1e-4


OBS_CHANNELS = 10  # revealed + nine count planes (env.py:80-85)
_OUTCOME_NAMES = {0: None, 1: "win", 2: "loss"}


class _LazyInfos(Mapping):
    """infos = {"aux": [...], "outcome": [...], "done": [...]} built on first access."""

    def __init__(self, step, last_new, frac, outcome, done):
        self._t = (step, last_new, frac, outcome, done)
        self._d: Optional[Dict[str, Any]] = None

    def _materialise(self):
        if self._d is None:
            step, last_new, frac, outcome, done = (t.cpu().numpy() for t in self._t)
            self._d = {
                "aux": [{"step": int(s), "last_new_reveals": int(n), "revealed_frac": float(f)}
                        for s, n, f in zip(step, last_new, frac)],
                "outcome": [_OUTCOME_NAMES[int(o)] for o in outcome],
                "done": [bool(x) for x in done],
            }
        return self._d

    def __getitem__(self, k):
        return self._materialise()[k]

    def __iter__(self):
        return iter(("aux", "outcome", "done"))

    def __len__(self):
        return 3

    # raw device tensors, for callers that want to stay on device
    @property
    def tensors(self) -> Dict[str, torch.Tensor]:
        step, last_new, frac, outcome, done = self._t
        return {"step": step, "last_new_reveals": last_new, "revealed_frac": frac,
                "outcome": outcome, "done": done}


class _EnvProxy:
    """Read-only stand-in for one MinesweeperEnv (H, W, cfg, revealed, flags,
    mine_mask, adjacent_counts, first_click_done, step_count), backed by
    ms_snapshot of the whole shard, cached until the next step/reset."""

    def __init__(self, vec: "VecMinesweeper", i: int):
        self._vec, self._i = vec, i
        self.cfg = vec.cfg
        self.H, self.W = vec.H, vec.W
        self.cell_count = self.reveal_count = self.A = vec.H * vec.W

    def _s(self):
        return self._vec._snapshot()

    @property
    def revealed(self) -> np.ndarray:
        return self._s()["revealed"][self._i]

    @property
    def mine_mask(self) -> np.ndarray:
        return self._s()["mine"][self._i]

    @property
    def adjacent_counts(self) -> np.ndarray:
        return self._s()["counts"][self._i]

    @property
    def flags(self) -> np.ndarray:  # never set on any reference path (env.py:246-276 has no callers)
        return np.zeros((self.H, self.W), dtype=bool)

    @property
    def first_click_done(self) -> bool:
        return bool(self._s()["first_click"][self._i])

    @property
    def step_count(self) -> int:
        return int(self._s()["step_count"][self._i])

    @property
    def action_space(self) -> int:
        return self.A

    @property
    def obs_channels(self) -> int:
        return OBS_CHANNELS


class _EnvList:
    def __init__(self, vec):
        self._vec = vec

    def __len__(self):
        return self._vec.num_envs

    def __getitem__(self, i):
        n = self._vec.num_envs
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(n))]
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError(i)
        return _EnvProxy(self._vec, i)

    def __iter__(self):
        return (self[i] for i in range(len(self)))


LATE_MODES = {"shared": 0, "keyed": 1}  # MS_LATE_SHARED / MS_LATE_KEYED


class VecMinesweeper:
    """Batched Minesweeper with all board state in HBM (one HIP handle)."""

    def __init__(self, num_envs: int, cfg: EnvConfig, seed: int = 0,
                 late_start_cfg: Optional[Dict[str, Any]] = None,
                 late_start_seed: Optional[int] = None, *, device=None,
                 shard: Tuple[int, int] = (0, 1), as_numpy: bool = False):
        assert num_envs > 0  # env.py:390
        rank, world = shard
        assert 0 <= rank < world and world <= num_envs
        self.cfg = cfg
        self.num_envs_total = int(num_envs)
        begin = self.num_envs_total * rank // world
        end = self.num_envs_total * (rank + 1) // world
        self.env_begin = begin
        self.num_envs = end - begin
        self.H, self.W = int(cfg.H), int(cfg.W)
        self.A = self.H * self.W
        self.as_numpy = as_numpy
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise L.MsEnvError("VecMinesweeper runs on a HIP device only (no CPU backend)")
        self._lib = L.load()
        c = L.MsCfg(self.H, self.W, int(cfg.mine_count), int(bool(cfg.guarantee_safe_neighborhood)),
                    float(cfg.win_reward), float(cfg.loss_reward), float(cfg.step_penalty))
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            L.check(self._lib.ms_create(ctypes.byref(c), self.num_envs_total, int(seed), begin,
                                        self.num_envs, ctypes.byref(h)))
        self._h = h
        # late start (env.py:397-403): one generator for all envs, seeded late_start_seed
        # or, as the reference, with the base generator's next draw after the N seeds
        self._late_start_cfg = dict(late_start_cfg) if late_start_cfg else None
        if self._late_start_cfg:
            if late_start_seed is None:
                base = np.random.default_rng(seed)
                base.integers(0, 2**31 - 1, size=self.num_envs_total, dtype=np.int64)
                late_start_seed = int(base.integers(0, 2**31 - 1))
            ls = self._late_start_cfg
            mn = int(ls.get("min_hidden", 5))
            # ls["rng"]: "shared" (default) = the reference's one generator, consumed in env order by
            # one wave (bit-exact; a shard cannot replay the global stream and draws its own);
            # "keyed" = one stream per reset keyed by global env (MS_LATE_KEYED, include/msenv.h):
            # every reset of a step in parallel, and a shard's resets are the unsharded run's
            mode = ls.get("rng", "shared")
            if mode not in LATE_MODES:
                raise ValueError(f"late_start_cfg rng must be one of {sorted(LATE_MODES)}, got {mode!r}")
            keyed = LATE_MODES[mode] == L.MS_LATE_KEYED
            lseed = int(late_start_seed) if (world == 1 or keyed) else \
                (int(late_start_seed) * 1000003 + begin) % 2**63
            L.check(self._lib.ms_set_late_start(h, float(ls.get("prob", 0.0)), mn, int(ls.get("max_hidden", mn)),
                                                int(ls.get("max_attempts", 3)),
                                                int(ls.get("max_extra_steps", self.A)), lseed))
            L.check(self._lib.ms_set_late_start_mode(h, LATE_MODES[mode]))
        self._version = 0
        self._snap = None
        self._snap_version = -1
        self.envs = _EnvList(self)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and getattr(self, "_lib", None) is not None:
            self._lib.ms_destroy(h)
            self._h = None

    # ------------------------------------------------------------------ API
    def action_space(self) -> int:
        return self.A

    def obs_channels(self) -> int:
        return OBS_CHANNELS

    def _stream(self):
        return L.stream_ptr(self.device)

    def _alloc_obs(self):
        obs = torch.empty((self.num_envs, OBS_CHANNELS, self.H, self.W), dtype=torch.float32,
                          device=self.device)
        mask = torch.empty((self.num_envs, self.A), dtype=torch.bool, device=self.device)
        return obs, mask

    def _host(self, d):
        if not self.as_numpy:
            return d
        return {k: v.cpu().numpy() for k, v in d.items()}

    def reset(self, out: Optional[Dict[str, torch.Tensor]] = None) -> Dict[str, Any]:
        obs, mask = (out["obs"], out["action_mask"]) if out else self._alloc_obs()
        with torch.cuda.device(self.device):
            L.check(self._lib.ms_reset(self._h, L.ptr(obs), L.ptr(mask), self._stream()))
        self._version += 1
        return self._host({"obs": obs, "action_mask": mask})

    def _as_actions(self, actions):
        if isinstance(actions, np.ndarray):
            assert actions.shape == (self.num_envs,)  # env.py:480
            a = torch.from_numpy(np.ascontiguousarray(actions))
        elif isinstance(actions, torch.Tensor):
            assert tuple(actions.shape) == (self.num_envs,)
            a = actions
        else:
            a = torch.as_tensor(actions)
            assert tuple(a.shape) == (self.num_envs,)
        if a.dtype not in (torch.int64, torch.int32):
            a = a.to(torch.int64)
        return a.to(self.device, non_blocking=True).contiguous()

    def step(self, actions, out: Optional[Dict[str, torch.Tensor]] = None):
        a = self._as_actions(actions)
        n = self.num_envs
        codes = out.get("codes") if out is not None else None
        if codes is not None:  # the rollout buffer's u8 cell codes instead of the f32 obs (ms_step_codes)
            assert codes.dtype == torch.uint8 and codes.is_contiguous() and codes.numel() == n * self.H * self.W
            if out.get("obs") is not None:
                raise ValueError("step(out=...): give either 'obs' or 'codes', not both (codes replace the obs)")
            if self.as_numpy:
                raise ValueError("step(out=...): 'codes' is a device-buffer path; it cannot be used with as_numpy=True")
            a = a.to(torch.int64)
        if out is not None:
            obs, mask = out.get("obs"), out["action_mask"]
            rewards, dones = out["rewards"], out["dones"]
        else:
            obs, mask = self._alloc_obs()
            rewards = torch.empty(n, dtype=torch.float32, device=self.device)
            dones = torch.empty(n, dtype=torch.bool, device=self.device)
        step = torch.empty(n, dtype=torch.int32, device=self.device)
        last_new = torch.empty(n, dtype=torch.int32, device=self.device)
        frac = torch.empty(n, dtype=torch.float64, device=self.device)
        outcome = torch.empty(n, dtype=torch.int8, device=self.device)
        if codes is not None:
            fn, o = self._lib.ms_step_codes, codes
        else:
            fn, o = (self._lib.ms_step if a.dtype == torch.int64 else self._lib.ms_step_i32), obs
        with torch.cuda.device(self.device):
            L.check(fn(self._h, L.ptr(a), L.ptr(o), L.ptr(mask), L.ptr(rewards), L.ptr(dones),
                       L.ptr(step), L.ptr(last_new), L.ptr(frac), L.ptr(outcome), self._stream()))
        self._version += 1
        infos = _LazyInfos(step, last_new, frac, outcome, dones)
        batch = {"obs": obs, "action_mask": mask} if codes is None else {"codes": codes, "action_mask": mask}
        batch = self._host(batch)
        if self.as_numpy:
            return batch, rewards.cpu().numpy(), dones.cpu().numpy(), infos
        return batch, rewards, dones, infos

    # ------------------------------------------------------- device helpers
    def mine_labels(self, labels: Optional[torch.Tensor] = None, valid: Optional[torch.Tensor] = None):
        """collect_rollout's label capture (train_rl.py:203-219) on device."""
        if labels is None:
            labels = torch.empty((self.num_envs, self.H, self.W), dtype=torch.float32, device=self.device)
        if valid is None:
            valid = torch.empty((self.num_envs, self.H, self.W), dtype=torch.bool, device=self.device)
        with torch.cuda.device(self.device):
            L.check(self._lib.ms_labels(self._h, L.ptr(labels), L.ptr(valid), self._stream()))
        return labels, valid

    def tape_actions(self, t: int, mode: int = L.MS_TAPE_UNIFORM, out: Optional[torch.Tensor] = None):
        """Synthetic policy of SURVEY.md §8d (used by bench.py and the parity tests)."""
        if out is None:
            out = torch.empty(self.num_envs, dtype=torch.int64, device=self.device)
        with torch.cuda.device(self.device):
            L.check(self._lib.ms_tape_actions(self._h, int(t), int(mode), L.ptr(out), self._stream()))
        return out

    _RUN_KEYS = ("actions", "obs", "action_mask", "rewards", "dones", "step", "last_new_reveals",
                 "revealed_frac", "outcome")

    def run_tape(self, t0: int, T: int, mode: int = L.MS_TAPE_UNIFORM, slots: bool = True) -> Dict[str, torch.Tensor]:
        """T synthetic-policy steps (tape_actions(t) then step, t = t0 .. t0+T-1) in ONE launch
        (ms_run_tape: the boards stay in registers between steps). slots=True returns every
        step's outputs stacked [T, N, ...]; slots=False only the last step's [N, ...].
        Bit-exact with the loop; not available with late-start resets."""
        n, A, dev = self.num_envs, self.H * self.W, self.device
        lead = (int(T), n) if slots else (n,)
        dt = {"actions": torch.int64, "obs": torch.float32, "action_mask": torch.bool, "rewards": torch.float32,
              "dones": torch.bool, "step": torch.int32, "last_new_reveals": torch.int32,
              "revealed_frac": torch.float64, "outcome": torch.int8}
        tail = {"obs": (OBS_CHANNELS, self.H, self.W), "action_mask": (A,)}
        out = {k: torch.empty(lead + tail.get(k, ()), dtype=dt[k], device=dev) for k in self._RUN_KEYS}
        with torch.cuda.device(dev):
            L.check(self._lib.ms_run_tape(self._h, int(t0), int(T), int(mode), 1 if slots else 0,
                                          *(L.ptr(out[k]) for k in self._RUN_KEYS), self._stream()))
        self._version += 1
        return out

    def set_debug_flags(self, flags: int) -> None:
        """msenv_debug.h hooks (tests): e.g. L.MS_DBG_FORCE_SERIAL_PLACEMENT."""
        L.check(self._lib.ms_set_debug_flags(self._h, int(flags)))

    def late_rng_state(self) -> np.ndarray:
        """The shared late-start generator's state u64[6] (ms_rng_state layout)."""
        out = np.zeros(6, dtype=np.uint64)
        torch.cuda.synchronize(self.device)
        L.check(self._lib.ms_late_rng_state(self._h, out.ctypes.data))
        return out

    def rng_state(self) -> np.ndarray:
        out = torch.empty((self.num_envs, 6), dtype=torch.int64, device=self.device)
        with torch.cuda.device(self.device):
            L.check(self._lib.ms_rng_state(self._h, L.ptr(out), self._stream()))
        return out.cpu().numpy().view(np.uint64)

    def snapshot_tensors(self) -> Dict[str, torch.Tensor]:
        n, H, W = self.num_envs, self.H, self.W
        d = {
            "mine": torch.empty((n, H, W), dtype=torch.bool, device=self.device),
            "revealed": torch.empty((n, H, W), dtype=torch.bool, device=self.device),
            "counts": torch.empty((n, H, W), dtype=torch.uint8, device=self.device),
            "first_click": torch.empty(n, dtype=torch.bool, device=self.device),
            "step_count": torch.empty(n, dtype=torch.int32, device=self.device),
        }
        with torch.cuda.device(self.device):
            L.check(self._lib.ms_snapshot(self._h, L.ptr(d["mine"]), L.ptr(d["revealed"]),
                                          L.ptr(d["counts"]), L.ptr(d["first_click"]),
                                          L.ptr(d["step_count"]), self._stream()))
        return d

    def _snapshot(self):
        if self._snap_version != self._version:
            self._snap = {k: v.cpu().numpy() for k, v in self.snapshot_tensors().items()}
            self._snap_version = self._version
        return self._snap


__all__ = ["EnvConfig", "VecMinesweeper", "SolverPreset", "OBS_CHANNELS"]

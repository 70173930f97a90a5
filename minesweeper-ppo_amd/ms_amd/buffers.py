"""On-device rollout storage + GAE (reference: minesweeper/buffers.py:9-116).

Same API as the reference RolloutBuffer (``add``, ``compute_gae``,
``get_minibatches``; row index = t * num_envs + env). Additions for the
MI355X path:
  * ``slot(t)`` returns views of row block t, so the board step writes the
    next observation / mask / reward / done straight into the buffer
    (no per-step copy);
  * the mine-label planes are preallocated when requested (the reference
    allocates lazily on first use, buffers.py:60-75 — same contents);
  * ``compute_gae`` runs the ms_gae HIP kernel (one thread per env, reverse
    scan), bitwise equal to the reference's torch loop (f32 op order kept);
  * ``obs_codes=True`` stores each observation as its u8 cell codes [H, W]
    (ms_amd.fused.obs_encode: 0 hidden, 1 + k revealed with k adjacent mines)
    instead of the f32 one-hot [10, H, W]: 40x fewer bytes to hold and to gather
    per minibatch (2.7 GB -> 67 MB at 4096 envs x 64 steps on 16x16). The
    policy takes codes directly (CNNResidualPolicy.forward); the obs are exact.
"""
from __future__ import annotations

from typing import Dict, Iterator, Optional, Tuple

import numpy as np
import torch

from . import _lib as L


class Batch:
    """Attribute bag handed to ppo_update (the reference builds an anonymous
    ``type("Batch", ...)``, buffers.py:116)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def __contains__(self, k):
        return k in self.__dict__


class RolloutBuffer:
    def __init__(self, num_envs: int, steps: int, obs_shape: Tuple[int, int, int], action_dim: int,
                 device: torch.device, with_mine_labels: bool = False, obs_codes: bool = False):
        self.num_envs = num_envs
        self.steps = steps
        self.device = torch.device(device)
        B = num_envs * steps
        C, H, W = obs_shape
        self.obs_shape = obs_shape
        self.obs_codes = obs_codes
        if obs_codes:
            if C != 10:
                raise ValueError("obs_codes needs the env's 10-plane observation")
            if self.device.type != "cuda":
                raise L.MsEnvError("obs_codes buffers are encoded on the HIP device (mc_obs_encode)")
            self.obs = torch.zeros((B, H, W), dtype=torch.uint8, device=device)
        else:
            self.obs = torch.zeros((B, C, H, W), dtype=torch.float32, device=device)
        self.action_mask = torch.zeros((B, action_dim), dtype=torch.bool, device=device)
        self.actions = torch.zeros((B,), dtype=torch.long, device=device)
        self.logp = torch.zeros((B,), dtype=torch.float32, device=device)
        self.rewards = torch.zeros((B,), dtype=torch.float32, device=device)
        self.dones = torch.zeros((B,), dtype=torch.bool, device=device)
        self.values = torch.zeros((B,), dtype=torch.float32, device=device)
        self.advantages = torch.zeros((B,), dtype=torch.float32, device=device)
        self.returns = torch.zeros((B,), dtype=torch.float32, device=device)
        self.mine_labels: Optional[torch.Tensor] = None
        self.mine_valid: Optional[torch.Tensor] = None
        if with_mine_labels:
            self.mine_labels = torch.zeros((B, H, W), dtype=torch.float32, device=device)
            self.mine_valid = torch.zeros((B, H, W), dtype=torch.bool, device=device)
        self._t = 0
        # this buffer's envs within the global env list (set by collect_rollout for a shard):
        # buffer row t*num_envs + e is global sample t*num_envs_total + env_begin + e
        self.env_begin = 0
        self.num_envs_total = num_envs

    # --------------------------------------------------------------- writes
    def slot(self, t: int) -> Dict[str, torch.Tensor]:
        s, e = t * self.num_envs, (t + 1) * self.num_envs
        d = {"obs": self.obs[s:e], "action_mask": self.action_mask[s:e], "actions": self.actions[s:e],
             "logp": self.logp[s:e], "rewards": self.rewards[s:e], "dones": self.dones[s:e],
             "values": self.values[s:e]}
        if self.mine_labels is not None:
            d["mine_labels"] = self.mine_labels[s:e]
            d["mine_valid"] = self.mine_valid[s:e]
        return d

    def add(self, obs, action_mask, actions, logp, rewards, dones, values,
            mine_labels: torch.Tensor | None = None, mine_valid: torch.Tensor | None = None) -> None:
        """buffers.py:38-76 (copying form, for callers that hold separate tensors)."""
        bsz = obs.shape[0]
        s, e = self._t * bsz, (self._t + 1) * bsz
        if self.obs_codes and obs.dtype != torch.uint8:
            from .fused import obs_encode
            obs_encode(obs.to(device=self.device, dtype=torch.float32).contiguous(), self.obs[s:e])
        else:
            self.obs[s:e] = obs
        self.action_mask[s:e] = action_mask
        self.actions[s:e] = actions
        self.logp[s:e] = logp
        self.rewards[s:e] = rewards
        self.dones[s:e] = dones
        self.values[s:e] = values
        if mine_labels is not None:
            if self.mine_labels is None:
                H, W = obs.shape[-2], obs.shape[-1]
                B = self.num_envs * self.steps
                self.mine_labels = torch.zeros((B, H, W), dtype=torch.float32, device=self.device)
            self.mine_labels[s:e] = mine_labels
            if mine_valid is not None:
                if self.mine_valid is None:
                    H, W = obs.shape[-2], obs.shape[-1]
                    B = self.num_envs * self.steps
                    self.mine_valid = torch.zeros((B, H, W), dtype=torch.bool, device=self.device)
                self.mine_valid[s:e] = mine_valid
        self._t += 1

    # ------------------------------------------------------------------ GAE
    def compute_gae(self, last_values: torch.Tensor, gamma: float = 0.995, lam: float = 0.95) -> None:
        """buffers.py:78-94 on the ms_gae kernel. gamma*lam is formed in double
        and rounded once, as `gamma * lam * next_non_terminal` does in torch."""
        if self.device.type != "cuda":
            raise L.MsEnvError("compute_gae runs on the HIP device only")
        lib = L.load()
        lv = last_values.detach().to(device=self.device, dtype=torch.float32).contiguous()
        dones_u8 = self.dones.view(torch.uint8)
        with torch.cuda.device(self.device):
            L.check(lib.ms_gae(L.ptr(self.rewards), L.ptr(self.values), L.ptr(dones_u8), L.ptr(lv),
                               self.steps, self.num_envs, float(np.float32(gamma)),
                               float(np.float32(gamma * lam)), L.ptr(self.advantages), L.ptr(self.returns),
                               L.stream_ptr(self.device)))

    # ----------------------------------------------------------- minibatches
    def get_minibatches(self, batch_size: int, generator: torch.Generator | None = None) -> Iterator[Batch]:
        """buffers.py:96-116: one device randperm per epoch, slices of batch_size."""
        B = self.obs.shape[0]
        idx = torch.randperm(B, device=self.device, generator=generator)
        for s in range(0, B, batch_size):
            yield self._gather(idx[s:s + batch_size])

    def get_stratified_minibatches(self, mini_batches: int, stripes: int, stripe_begin: int,
                                   seed: int) -> Iterator[Batch]:
        """World-invariant minibatches for data-parallel training. The GLOBAL env list is cut
        into stripes of equal size; this buffer holds ``stripes`` of them, starting at global
        stripe ``stripe_begin``. Each stripe's T*n_s rows get their own permutation, seeded by
        (seed, global stripe), and minibatch k takes slice k of every stripe's permutation.
        So minibatch k of a rank is exactly its part of minibatch k of an unsharded run with
        the same seed, and all ranks hold equal row counts (the mean of the rank means is the
        global mean). Compared with buffers.py:96-116's one randperm(B), every minibatch is
        stratified over env stripes: it holds the same number of rows from each stripe."""
        N, T = self.num_envs, self.steps
        assert N % stripes == 0, "envs must split evenly into stripes"
        n_s = N // stripes
        rows_s = T * n_s
        m_s = max(1, rows_s // mini_batches)
        perms = []
        for j in range(stripes):
            g = torch.Generator(device=self.device)
            g.manual_seed(_mix64(seed, stripe_begin + j))
            q = torch.randperm(rows_s, device=self.device, generator=g)
            perms.append((q // n_s) * N + j * n_s + (q % n_s))  # stripe row -> buffer row t*N + e
        P = torch.stack(perms)
        for s in range(0, rows_s, m_s):
            yield self._gather(P[:, s:s + m_s].reshape(-1))

    def global_rows(self, sel: torch.Tensor) -> torch.Tensor:
        """Buffer rows -> global sample ids t * num_envs_total + env_begin + e."""
        return (sel // self.num_envs) * self.num_envs_total + self.env_begin + sel % self.num_envs

    def _gather(self, sel: torch.Tensor) -> Batch:
        kw = dict(obs=self.obs[sel], action_mask=self.action_mask[sel], actions=self.actions[sel],
                  old_logp=self.logp[sel], rewards=self.rewards[sel], dones=self.dones[sel],
                  values=self.values[sel], advantages=self.advantages[sel], returns=self.returns[sel],
                  rows=self.global_rows(sel))
        if self.mine_labels is not None:
            kw["mine_labels"] = self.mine_labels[sel]
            if self.mine_valid is not None:
                kw["mine_valid"] = self.mine_valid[sel]
        return Batch(**kw)


def _mix64(a: int, b: int) -> int:
    """splitmix64 finaliser of (a, b) -> a 63-bit generator seed."""
    M = (1 << 64) - 1
    z = (a * 0x9E3779B97F4A7C15 + b + 0x632BE59BD9B4E019) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return (z ^ (z >> 31)) >> 1


__all__ = ["RolloutBuffer", "Batch"]

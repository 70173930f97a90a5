"""Dropout2d masks keyed by global sample index (ms_dropout_masks, include/msenv.h).

The reference draws its Dropout2d masks (cnn_residual.py:14,22) from torch's global RNG
in every training-mode forward: the rollout forward (train_rl.py:221) and each
minibatch forward of ppo_update (ppo.py:25-30). Under data parallelism a shared torch
seed would give every rank the same masks for its local rows, and a per-rank seed
would give masks that depend on the world size. Here a mask is a counter-based hash of
(seed, counter, GLOBAL sample id, block, channel): the sample at buffer row
t * num_envs_total + global_env draws the same masks whichever rank holds it, so the
data-parallel update is the one-GPU update (tests/test_dist_trainer_gpu.py).

Use::

    with keyed_dropout(model, rows, seed, counter):
        logits, value = model(obs)          # rows: int64 [N] global sample ids

Without a key (standalone calls), the model falls back to torch-RNG masks.
"""
from __future__ import annotations

from contextlib import contextmanager

import torch

from . import _lib as L

# key domains: the rollout forward and the minibatch forwards draw from disjoint streams
ROLLOUT, MINIBATCH = 1, 2


def dropout_masks(rows: torch.Tensor, nblk: int, channels: int, p: float, seed: int, counter: int) -> torch.Tensor:
    """f32 [nblk, N, channels]: keep / (1 - p) per (block, sample, channel)."""
    lib = L.load()
    rows = rows.to(torch.int64).contiguous()
    n = rows.shape[0]
    out = torch.empty((nblk, n, channels), dtype=torch.float32, device=rows.device)
    L.check(lib.ms_dropout_masks(L.ptr(rows), n, nblk, channels, int(seed) & (2**64 - 1),
                                 int(counter) & (2**64 - 1), float(p), L.ptr(out), L.stream_ptr(rows.device)))
    return out


@contextmanager
def keyed_dropout(model: torch.nn.Module, rows: torch.Tensor | None, seed: int, counter: int):
    """Within the block, ``model``'s training-mode forwards draw keyed masks for ``rows``."""
    prev = getattr(model, "_dropout_key", None)
    model._dropout_key = None if rows is None else (rows, int(seed), int(counter))
    try:
        yield
    finally:
        model._dropout_key = prev


def mix_seed(seed: int, domain: int) -> int:
    """splitmix64 of (seed, domain): the per-domain hash seed."""
    M = (1 << 64) - 1
    z = (int(seed) * 0x9E3779B97F4A7C15 + domain * 0xD6E8FEB86659FD93 + 0x632BE59BD9B4E019) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


__all__ = ["dropout_masks", "keyed_dropout", "mix_seed", "ROLLOUT", "MINIBATCH"]

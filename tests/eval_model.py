"""A deterministic stand-in policy for evaluation parity tests (our code, shared by
tests/golden/gen_eval_golden.py and tests/test_eval.py).

Logits and mine logits are exact in fp32 on any device: small integer neighbourhood
sums of the observation plus a per-cell fraction k/1024 that makes every cell's logit
distinct (no argmax ties)."""
import torch
import torch.nn as nn


def _nsum(x):  # 3x3 neighbourhood sum with zero padding, elementwise adds only
    p = torch.nn.functional.pad(x, (1, 1, 1, 1))
    H, W = x.shape[-2:]
    return sum(p[..., dy:dy + H, dx:dx + W] for dy in range(3) for dx in range(3))


class DetModel(nn.Module):
    def __init__(self):
        super().__init__()
        self.dummy = nn.Parameter(torch.zeros(1))

    def forward(self, obs, return_mine=False):
        n, _, H, W = obs.shape
        rev = obs[:, 0]
        cnt = (obs[:, 1:10] * torch.arange(9, dtype=obs.dtype, device=obs.device)[None, :, None, None]).sum(1)
        nrev, ncnt = _nsum(rev), _nsum(cnt)
        idx = torch.arange(H * W, dtype=obs.dtype, device=obs.device).view(1, H, W)
        frac = torch.remainder(idx * 37.0, 1024.0) / 1024.0
        logits = (nrev * 2.0 - ncnt * 3.0 + frac).reshape(n, -1) + self.dummy * 0
        value = logits.mean(1) * 0.0
        if not return_mine:
            return logits, value
        mine = ((ncnt - nrev) * 0.5 + frac * 0.25)[:, None]
        return logits, value, mine


class RuleModel(nn.Module):
    """Deterministic single-point-rule player, exact in fp32 on any device (small integer
    neighbourhood sums, equality tests, and the same per-cell k/1024 tie-breaker), strong
    enough to WIN 16x16x40 and 30x16x99 boards now and then, so evaluation fixtures cover
    win accounting and a meaningful belief AUROC:
      hidden neighbours h and count c of every revealed cell;
      certain mines: hidden cells next to a revealed cell with c == h > 0;
      certain safe: other hidden cells next to a revealed cell whose c equals its number of
      certain-mine neighbours.
    Logits prefer certain-safe cells, then the DetModel guess heuristic; mine logits rank
    certain mines above unknowns above certain-safe cells."""

    def __init__(self):
        super().__init__()
        self.dummy = nn.Parameter(torch.zeros(1))

    def forward(self, obs, return_mine=False):
        n, _, H, W = obs.shape
        rev = obs[:, 0]
        hid = 1.0 - rev
        cnt = (obs[:, 1:10] * torch.arange(9, dtype=obs.dtype, device=obs.device)[None, :, None, None]).sum(1)
        h = _nsum(hid) * rev
        full = rev * (cnt == h).to(obs.dtype) * (h > 0).to(obs.dtype)
        mine = hid * (_nsum(full) > 0).to(obs.dtype)
        m = _nsum(mine) * rev
        done = rev * (cnt == m).to(obs.dtype)
        safe = hid * (1.0 - mine) * (_nsum(done) > 0).to(obs.dtype)
        nrev, ncnt = _nsum(rev), _nsum(cnt)
        idx = torch.arange(H * W, dtype=obs.dtype, device=obs.device).view(1, H, W)
        frac = torch.remainder(idx * 37.0, 1024.0) / 1024.0
        logits = (safe * 256.0 - mine * 256.0 + nrev * 2.0 - ncnt * 3.0 + frac).reshape(n, -1) + self.dummy * 0
        value = logits.mean(1) * 0.0
        if not return_mine:
            return logits, value
        ml = (mine * 8.0 - safe * 8.0 + (ncnt - nrev) * 0.5 + frac * 0.25)[:, None]
        return logits, value, ml

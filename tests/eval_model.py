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

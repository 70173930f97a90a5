"""On-device rollout collection (reference: train_rl.py:155-289, collect_rollout).

Per step, everything stays in HBM on one stream:
  ms_labels  -> buffer.mine_labels/mine_valid[t]   (labels of obs_t, train_rl.py:203-219)
  model fwd  -> logits, values                     (autocast, train_rl.py:221-227)
  ms_sample_masked -> buffer.actions[t], logp[t]   (masked Categorical, train_rl.py:229-235)
  ms_step    -> buffer.obs/mask[t+1], rewards[t], dones[t]  (env.step, train_rl.py:242)
There is no host round trip inside the loop (the reference crosses the PCIe
boundary three times per step, train_rl.py:198-199, 239, 246-247).

Sampling is Gumbel-max over the valid cells from a counter-based hash, so the
action distribution equals softmax(masked logits) (checked statistically in
tests); the stream of random numbers is not torch's, hence rollouts are not
bitwise those of torch.distributions.Categorical. The hash is keyed by the
GLOBAL env index, so a rank's shard draws what the same envs draw in an
unsharded run: rollouts do not depend on the world size. The training-mode
forward's Dropout2d masks are keyed the same way (ms_amd.dropout).
"""
from __future__ import annotations

import time
from contextlib import nullcontext
from typing import Dict, Optional, Tuple

import torch

from . import _lib as L
from .buffers import RolloutBuffer
from .dropout import ROLLOUT, keyed_dropout, mix_seed
from .env import OBS_CHANNELS, VecMinesweeper
from .profiling import PhaseTimer, RolloutTimings, prange


def sample_masked(logits: torch.Tensor, mask: torch.Tensor, seed: int, counter: int,
                  actions: Optional[torch.Tensor] = None, logp: Optional[torch.Tensor] = None,
                  row_begin: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Categorical(logits.masked_fill(~mask, -inf)).sample() + log_prob on device. Row i draws
    from the hash stream of global row ``row_begin + i``."""
    lib = L.load()
    lg = logits.detach().float().contiguous()
    n, a = lg.shape
    if actions is None:
        actions = torch.empty(n, dtype=torch.int64, device=lg.device)
    if logp is None:
        logp = torch.empty(n, dtype=torch.float32, device=lg.device)
    m = mask.contiguous().view(torch.uint8)
    L.check(lib.ms_sample_masked(L.ptr(lg), L.ptr(m), n, a, int(row_begin), int(seed) & (2**64 - 1),
                                 int(counter) & (2**64 - 1), L.ptr(actions), L.ptr(logp),
                                 L.stream_ptr(lg.device)))
    return actions, logp


def _autocast(device: torch.device, amp_dtype):
    if device.type == "cuda" and amp_dtype is not None:
        return torch.autocast(device_type="cuda", dtype=amp_dtype)
    return nullcontext()


@torch.no_grad()
def collect_rollout(vec: VecMinesweeper, model: torch.nn.Module, steps: int, device: torch.device,
                    aux_mine_weight: float = 0.0, aux_mine_calib_weight: float = 0.0, *,
                    amp_dtype: Optional[torch.dtype] = torch.bfloat16, buffer: Optional[RolloutBuffer] = None,
                    sample_seed: int = 0, sample_counter: int = 0, obs_codes: bool = False, timing: bool = True
                    ) -> Tuple[RolloutBuffer, Dict]:
    """Same contract as the reference: returns (buffer, {"last_values", "timings"}); ``timings`` has
    the reference's keys (train_rl.py:278-288), timed on the GPU with HIP events and resolved (one
    host sync) on first read (ms_amd.profiling.RolloutTimings); ``timing=False`` records no events.
    ``buffer`` may be passed back in to reuse its HBM (2.7 GB at N=4096, T=64; 67 MB with
    ``obs_codes``: the buffer then holds u8 cell codes, which the env step writes directly
    (ms_step_codes); only the reset obs and the last step's obs pass through f32)."""
    device = torch.device(device)
    need_aux = aux_mine_weight > 0 or aux_mine_calib_weight > 0
    N, H, W = vec.num_envs, vec.H, vec.W
    if buffer is None or buffer.num_envs != N or buffer.steps != steps or \
            (need_aux and buffer.mine_labels is None) or buffer.obs_codes != obs_codes:
        buffer = RolloutBuffer(N, steps, (OBS_CHANNELS, H, W), H * W, device, with_mine_labels=need_aux,
                               obs_codes=obs_codes)
    if buffer.obs_codes:
        from .fused import obs_encode
    # global sample ids (row t * num_envs_total + global env): keys of the Dropout2d masks
    buffer.env_begin, buffer.num_envs_total = vec.env_begin, vec.num_envs_total
    env_ids = torch.arange(vec.env_begin, vec.env_begin + N, dtype=torch.int64, device=device)
    dseed = mix_seed(sample_seed, ROLLOUT)
    t0 = time.perf_counter()
    tm = PhaseTimer(device, enabled=timing)
    s0 = buffer.slot(0)
    last_obs = torch.empty((N, OBS_CHANNELS, H, W), dtype=torch.float32, device=device)
    last_mask = torch.empty((N, H * W), dtype=torch.bool, device=device)
    # codes mode: the reset obs goes through last_obs (f32) and is encoded into slot 0
    vec.reset(out={"obs": last_obs if buffer.obs_codes else s0["obs"], "action_mask": s0["action_mask"]})
    if buffer.obs_codes:
        obs_encode(last_obs, s0["obs"])
    tm.start()
    for t in range(steps):
        s = buffer.slot(t)
        if need_aux:
            with prange("rollout/labels"):
                vec.mine_labels(s["mine_labels"], s["mine_valid"])
            tm.split("mine_label_copy")
        with prange("rollout/forward"):
            with _autocast(device, amp_dtype), \
                    keyed_dropout(model, env_ids + t * vec.num_envs_total, dseed, sample_counter + t):
                logits, values = model(s["obs"])
            sample_masked(logits, s["action_mask"], sample_seed, sample_counter + t, s["actions"], s["logp"],
                          row_begin=vec.env_begin)
        tm.split("model_forward")
        s["values"].copy_(values.float())
        tm.split("tensor_bridge")
        if t + 1 < steps:
            nxt = buffer.slot(t + 1)
            # codes buffer: the env writes the next step's cell codes straight into it (ms_step_codes)
            out = ({"codes": nxt["obs"], "action_mask": nxt["action_mask"]} if buffer.obs_codes else
                   {"obs": nxt["obs"], "action_mask": nxt["action_mask"]})
        else:
            out = {"obs": last_obs, "action_mask": last_mask}
        out["rewards"], out["dones"] = s["rewards"], s["dones"]
        with prange("rollout/env_step"):
            vec.step(s["actions"], out=out)
        tm.split("env_step")
    with prange("rollout/bootstrap"), _autocast(device, amp_dtype), \
            keyed_dropout(model, env_ids + steps * vec.num_envs_total, dseed, sample_counter + steps):
        _, last_values = model(last_obs)
    last_values = last_values.float()
    buffer._t = steps
    timings = RolloutTimings(steps, tm, time.perf_counter() - t0)
    return buffer, {"last_values": last_values, "timings": timings, "last_obs": last_obs,
                    "last_mask": last_mask}


__all__ = ["collect_rollout", "sample_masked"]

"""PPO loss + update (reference: minesweeper/ppo.py:11-119).

Same losses and order of operations: masked log-softmax, clipped policy
ratio, clipped value loss (0.5 * max), entropy bonus, optional belief BCE
(pos_weight = neg/pos over the valid cells of the minibatch) and calibration
MSE, then backward, unscale, clip_grad_norm_(max_grad_norm), optimizer step.

Data-parallel form (``group`` given, one process per GPU over RCCL): every
rank holds an equal slice of the global minibatch. Row-mean losses are then
exactly the global ones after gradient averaging; the belief BCE/MSE, whose
denominator is the global count of valid cells, is computed as
local_sum * world / global_count after one 2-float all-reduce of (pos, count),
and pos_weight uses the global counts — so an N-rank update equals the
single-device update on the concatenated minibatch up to summation order.
Gradients are averaged with ONE all-reduce over a flat bucket (FlatGrads).
"""
from __future__ import annotations

import weakref
from contextlib import nullcontext
from dataclasses import dataclass
from typing import Dict, Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import loss as _loss
from .profiling import prange


@dataclass
class PPOConfig:
    clip_eps: float = 0.2
    clip_eps_v: float = 0.2
    vf_coef: float = 0.5
    ent_coef: float = 0.003
    aux_mine_weight: float = 0.0
    aux_mine_calib_weight: float = 0.0
    max_grad_norm: float = 0.5
    beta_l2: float = 0.0


class FlatGrads:
    """All parameter gradients as views of one contiguous buffer, so the
    data-parallel reduction is a single RCCL all-reduce (3.80 MB for the
    shipped 950,947-parameter model) instead of one per tensor.

    A post-accumulate hook records which parameters the backward reached.
    ``release_unused()`` sets ``.grad = None`` on the others (e.g. the mine
    head when both belief-loss weights are 0), so the optimizer skips them as
    it does after the reference's ``zero_grad(set_to_none=True)``
    (ppo.py:96): no weight decay, no momentum step on a stale gradient."""

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.reached = set()
        # the hooks hold only a weak reference: a dropped FlatGrads (and its flat buffer) is
        # freed, and its hooks are removed by the finaliser or by close()
        ref = weakref.ref(self)

        def mark(p, ref=ref):
            me = ref()
            if me is not None:
                me.reached.add(id(p))
        self._handles = [p.register_post_accumulate_grad_hook(mark) for p in self.params]
        self._finalizer = weakref.finalize(self, _remove_hooks, self._handles)
        self.attach()

    def close(self):
        """Remove the hooks (the gradients stay as they are)."""
        self._finalizer()

    def attach(self):
        o = 0
        for p in self.params:
            k = p.numel()
            p.grad = self.flat[o:o + k].view_as(p)
            o += k

    def zero(self):
        self.flat.zero_()
        self.reached.clear()
        # an optimizer's zero_grad(set_to_none=True) or autograd may have replaced .grad
        for p in self.params:
            if p.grad is None or p.grad.data_ptr() < self.flat.data_ptr() or \
                    p.grad.data_ptr() >= self.flat.data_ptr() + self.flat.numel() * 4:
                self.attach()
                break

    def release_unused(self):
        """After backward: parameters no gradient reached get ``.grad = None``
        (``zero()`` re-attaches the views). Which parameters are reached
        depends only on the loss configuration, so it agrees across ranks."""
        for p in self.params:
            if id(p) not in self.reached:
                p.grad = None

    def all_reduce_mean(self, group=None):
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
        self.flat.div_(dist.get_world_size(group))


def _remove_hooks(handles):
    for h in handles:
        h.remove()
    handles.clear()


def _autocast(batch_obs: torch.Tensor, amp_dtype: Optional[torch.dtype]):
    if batch_obs.is_cuda and amp_dtype is not None:
        return torch.autocast(device_type="cuda", dtype=amp_dtype)
    return nullcontext()


def ppo_losses(model, batch, cfg: PPOConfig, amp_dtype: Optional[torch.dtype] = torch.bfloat16,
               group=None) -> Dict[str, torch.Tensor]:
    """Forward + losses (ppo.py:24-94). Returns 0-dim tensors (no host sync)."""
    world = dist.get_world_size(group) if group is not None else 1
    with _autocast(batch.obs, amp_dtype):
        need_mine = cfg.aux_mine_weight > 0 or cfg.aux_mine_calib_weight > 0
        if need_mine:
            logits, value, mine_logits = model(batch.obs, return_mine=True)
        else:
            logits, value = model(batch.obs, return_mine=False)
            mine_logits = None
        if logits.is_cuda and _loss.FUSED_LOSS and logits.shape[-1] <= 512:
            return _fused_losses(model, batch, cfg, amp_dtype, group, world, logits, value,
                                 mine_logits if need_mine else None)
        neg_inf = -1e4 if logits.dtype in (torch.float16, torch.bfloat16) else -1e9
        masked = logits.masked_fill(~batch.action_mask, neg_inf)
        logp = F.log_softmax(masked, dim=-1)
        logp_act = logp.gather(1, batch.actions.unsqueeze(1)).squeeze(1)
        ratio = (logp_act - batch.old_logp).exp()
        s1 = ratio * batch.advantages
        s2 = torch.clamp(ratio, 1 - cfg.clip_eps, 1 + cfg.clip_eps) * batch.advantages
        policy_loss = -torch.min(s1, s2).mean()
        vpred = value.view(-1)
        vclip = batch.values + (vpred - batch.values).clamp(-cfg.clip_eps_v, cfg.clip_eps_v)
        value_loss = 0.5 * torch.max((vpred - batch.returns).pow(2), (vclip - batch.returns).pow(2)).mean()
        ent = -(torch.softmax(masked, -1) * logp).sum(-1).mean()
        loss = policy_loss + cfg.vf_coef * value_loss - cfg.ent_coef * ent
        out = {"policy_loss": policy_loss, "value_loss": value_loss, "entropy": ent}
        if need_mine and getattr(batch, "mine_labels", None) is not None and mine_logits is not None:
            # masked sums instead of boolean gathers: no host sync (the reference's
            # lf[mask] + float(pos_weight) sync twice per minibatch, ppo.py:64-71)
            # under 16-bit autocast the reference's mine logits are 16-bit tensors: its pos_weight is
            # rounded to their dtype (ppo.py:70) and its calibration sigmoid runs in it (ppo.py:78-79)
            amp16 = batch.obs.is_cuda and amp_dtype in (torch.float16, torch.bfloat16)
            lf16 = mine_logits.squeeze(1).to(amp_dtype) if amp16 else mine_logits.squeeze(1)
            lf = lf16.float()
            y = batch.mine_labels
            vmask = getattr(batch, "mine_valid", None)
            vm = torch.ones_like(y) if vmask is None else vmask.to(y.dtype)
            pc = torch.stack([(y * vm).sum(), vm.sum()])
            if group is not None:
                dist.all_reduce(pc, group=group)
            pos, cnt = pc[0], pc[1]
            scale = world / cnt.clamp_min(1.0)  # empty valid set -> 0 loss (ppo.py:82-87)
            if cfg.aux_mine_weight > 0:
                pw = (cnt - pos + 1e-6) / (pos + 1e-6)
                if amp16:
                    pw = pw.to(amp_dtype).float()
                bce = F.binary_cross_entropy_with_logits(lf, y, pos_weight=pw, reduction="none")
                aux_bce = (bce * vm).sum() * scale
                loss = loss + cfg.aux_mine_weight * aux_bce
                out["aux_bce"] = aux_bce
            if cfg.aux_mine_calib_weight > 0:
                calib = ((torch.sigmoid(lf16).float() - y).pow(2) * vm).sum() * scale
                loss = loss + cfg.aux_mine_calib_weight * calib
                out["aux_calib"] = calib
        if cfg.beta_l2 > 0 and hasattr(model, "beta_regularizer"):
            loss = loss + cfg.beta_l2 * model.beta_regularizer()
        out["loss"] = loss
    return out


def _fused_losses(model, batch, cfg, amp_dtype, group, world, logits, value, mine_logits):
    """ppo_losses' terms from csrc/msppo.hip (ms_amd/loss.py): the same quantities, roundings
    and global belief counts, in one HIP pass forward and one backward (ppo.py:33-87)."""
    ml = mine_logits if (mine_logits is not None and getattr(batch, "mine_labels", None) is not None) else None
    counts = None
    if ml is not None:
        y = batch.mine_labels
        vmask = getattr(batch, "mine_valid", None)
        vm = torch.ones_like(y) if vmask is None else vmask.to(y.dtype)
        counts = torch.stack([(y * vm).sum(), vm.sum()])
        if group is not None:
            dist.all_reduce(counts, group=group)
    amp16 = amp_dtype if (batch.obs.is_cuda and amp_dtype in (torch.float16, torch.bfloat16)) else None
    t = _loss.ppo_loss_terms(logits, value, ml, batch, cfg, counts, world, amp16)
    out = {"policy_loss": t[0], "value_loss": t[1], "entropy": t[2]}
    if ml is not None:
        if cfg.aux_mine_weight > 0:
            out["aux_bce"] = t[3]
        if cfg.aux_mine_calib_weight > 0:
            out["aux_calib"] = t[4]
    loss = t[5]
    if cfg.beta_l2 > 0 and hasattr(model, "beta_regularizer"):
        loss = loss + cfg.beta_l2 * model.beta_regularizer()
    out["loss"] = loss
    return out


def ppo_update(model, optimizer, batch, cfg: PPOConfig, scaler=None, *,
               amp_dtype: Optional[torch.dtype] = torch.bfloat16, group=None,
               flat_grads: Optional[FlatGrads] = None, sync_stats: bool = True):
    """One minibatch update (ppo.py:23-119). With ``sync_stats=False`` the
    stats stay on device (0-dim tensors) so a caller can average them over an
    update with a single host sync. A data-parallel call (``group``) needs
    ``flat_grads``: the gradient all-reduce runs over its flat bucket."""
    if group is not None and flat_grads is None:
        raise ValueError("ppo_update(group=...) needs flat_grads=FlatGrads(model.parameters())")
    with prange("ppo/forward"):
        out = ppo_losses(model, batch, cfg, amp_dtype=amp_dtype, group=group)
    loss = out["loss"]
    if flat_grads is not None:
        flat_grads.zero()
    else:
        optimizer.zero_grad(set_to_none=True)
    if scaler is not None and batch.obs.is_cuda:
        with prange("ppo/backward"):
            scaler.scale(loss).backward()
        if flat_grads is not None:
            flat_grads.release_unused()
        if group is not None:
            with prange("ppo/all_reduce"):
                flat_grads.all_reduce_mean(group)
        with prange("ppo/optimizer"):
            scaler.unscale_(optimizer)
            torch.nn.utils.clip_grad_norm_(model.parameters(), cfg.max_grad_norm)
            scaler.step(optimizer)
            scaler.update()
    else:
        with prange("ppo/backward"):
            loss.backward()
        if flat_grads is not None:
            flat_grads.release_unused()
        if group is not None:
            with prange("ppo/all_reduce"):
                flat_grads.all_reduce_mean(group)
        with prange("ppo/optimizer"):
            torch.nn.utils.clip_grad_norm_(model.parameters(), cfg.max_grad_norm)
            optimizer.step()
    stats = {k: v.detach().float() for k, v in out.items()}
    if sync_stats:
        keys = sorted(stats)
        vals = torch.stack([stats[k] for k in keys]).tolist()
        return dict(zip(keys, vals))
    return stats


__all__ = ["PPOConfig", "FlatGrads", "ppo_losses", "ppo_update"]

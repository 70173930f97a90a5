"""The PPO minibatch loss on the GPU in two HIP passes (csrc/msppo.hip, C ABI include/msppo.h).

``ppo_loss_terms`` returns the reference's loss terms (minesweeper/ppo.py:33-87: policy, value,
entropy, belief BCE, calibration, and their weighted sum) as one f32 [8] tensor whose autograd
backward is the second pass: dlogits, dvalue and dmine in one launch instead of PyTorch's ~40
element-wise and reduction kernels each way. ms_amd/ppo.py ``ppo_losses`` takes this path on
CUDA (``FUSED_LOSS``; ``MS_FUSED_LOSS=0`` keeps the PyTorch ops, for A/B runs and parity tests).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

from . import _lib as L
from .fused import _check, _fn

FUSED_LOSS = os.environ.get("MS_FUSED_LOSS", "1") != "0"
MP_F32 = -1
_DT = {torch.float32: MP_F32, torch.bfloat16: 0, torch.float16: 1}  # MP_F32 / MC_DTYPE_BF16 / MC_DTYPE_F16
OUT_KEYS = ("policy_loss", "value_loss", "entropy", "aux_bce", "aux_calib", "loss")


class _Args(ctypes.Structure):
    """mc_ppo_loss_args (include/msppo.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("logits", "action_mask", "actions", "old_logp", "advantages",
                                                "values", "returns", "vpred", "mine", "labels", "valid",
                                                "counts")] + \
        [("vpred_dtype", ctypes.c_int32), ("mine_round", ctypes.c_int32)] + \
        [(n, ctypes.c_float) for n in ("clip_eps", "clip_eps_v", "vf_coef", "ent_coef", "aux_mine_weight",
                                       "aux_mine_calib_weight", "mask_fill", "world")] + \
        [("M", ctypes.c_int64), ("A", ctypes.c_int32)]


_fw = _bw = _ws = None


def _bind():
    global _fw, _bw, _ws
    if _fw is None:
        vp = ctypes.c_void_p
        _fw = _fn("mc_ppo_loss_fwd", [ctypes.POINTER(_Args), vp, vp, ctypes.c_int64, vp])
        _bw = _fn("mc_ppo_loss_bwd", [ctypes.POINTER(_Args), vp, vp, ctypes.c_int64, vp, vp, vp, vp])
        _ws = _fn("mc_ppo_loss_workspace", [ctypes.c_int64])
        _ws.restype = ctypes.c_int64


def _p(t: Optional[torch.Tensor]):
    return None if t is None else L.ptr(t)


class _LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, vpred, mine, keep, args):
        # keep: the non-differentiable row tensors the args point at (alive until backward)
        dev = logits.device
        out = torch.empty(8, dtype=torch.float32, device=dev)
        nws = int(_ws(args.M))
        work = torch.empty(nws, dtype=torch.float32, device=dev)
        _check(_fw(ctypes.byref(args), L.ptr(out), L.ptr(work), nws, L.stream_ptr(dev)))
        ctx.save_for_backward(logits, vpred, mine, work)
        ctx.keep, ctx.args = keep, args
        return out

    @staticmethod
    def backward(ctx, gout):
        logits, vpred, mine, work = ctx.saved_tensors
        gout = gout.float().contiguous()
        dl = torch.empty_like(logits)
        dv = torch.empty_like(vpred)
        dm = torch.empty_like(mine) if mine is not None else None
        _check(_bw(ctypes.byref(ctx.args), L.ptr(gout), L.ptr(work), work.numel(), L.ptr(dl), L.ptr(dv), _p(dm),
                   L.stream_ptr(logits.device)))
        return dl, dv, dm, None, None


def ppo_loss_terms(logits, value, mine_logits, batch, cfg, counts: Optional[torch.Tensor], world: int,
                   amp16: Optional[torch.dtype]) -> torch.Tensor:
    """f32 [8] = (policy_loss, value_loss, entropy, aux_bce, aux_calib, loss, 0, 0) as
    ms_amd/ppo.py ppo_losses computes them (ppo.py:33-87). ``mine_logits`` None: no belief terms;
    otherwise ``counts`` = global (sum labels * valid, sum valid). ``amp16``: the 16-bit autocast
    type the reference rounds the belief logits to, or None."""
    _bind()
    n = logits.shape[0]
    A = logits.shape[-1]
    mask_fill = -1e4 if logits.dtype in (torch.float16, torch.bfloat16) else -1e9
    lg = logits.float().contiguous()
    vp = value.reshape(-1)
    if vp.dtype not in _DT:
        vp = vp.float()
    vp = vp.contiguous()
    f32 = lambda t: t.detach().to(torch.float32).contiguous()  # noqa: E731
    keep = [batch.action_mask.contiguous(), batch.actions.to(torch.int64).contiguous(), f32(batch.old_logp),
            f32(batch.advantages), f32(batch.values), f32(batch.returns)]
    mine = None
    if mine_logits is not None:
        mine = mine_logits.reshape(n, -1).float().contiguous()
        vmask = getattr(batch, "mine_valid", None)
        keep += [f32(batch.mine_labels.reshape(n, -1)),
                 vmask.reshape(n, -1).contiguous() if vmask is not None else None, counts.float().contiguous()]
    else:
        keep += [None, None, None]
    if keep[0].dtype != torch.bool or (keep[7] is not None and keep[7].dtype != torch.bool):
        raise TypeError("action_mask and mine_valid must be torch.bool")
    a = _Args()
    (a.action_mask, a.actions, a.old_logp, a.advantages, a.values, a.returns, a.labels, a.valid, a.counts) = \
        [_p(t) for t in keep]
    a.logits, a.vpred, a.mine = L.ptr(lg), L.ptr(vp), _p(mine)
    a.vpred_dtype = _DT[vp.dtype]
    a.mine_round = _DT[amp16] if amp16 is not None else MP_F32
    a.clip_eps, a.clip_eps_v, a.vf_coef, a.ent_coef = cfg.clip_eps, cfg.clip_eps_v, cfg.vf_coef, cfg.ent_coef
    a.aux_mine_weight, a.aux_mine_calib_weight = cfg.aux_mine_weight, cfg.aux_mine_calib_weight
    a.mask_fill, a.world, a.M, a.A = mask_fill, float(world), n, A
    return _LossFn.apply(lg, vp, mine, keep, a)


__all__ = ["FUSED_LOSS", "OUT_KEYS", "ppo_loss_terms"]

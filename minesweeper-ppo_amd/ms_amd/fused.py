"""Fused MFMA residual-CNN layer ops (csrc/mscnn.hip, C ABI include/mscnn.h).

Activations are NHWC [N, H*W, C] in a 16-bit type: bf16 (bf16 autocast) or fp16 (fp16
autocast, the reference's training precision, ppo.py:25); weights are re-laid out as
[9, 96, CIN] (tap-major) of the same type. These ops replace, for CNNResidualPolicy
(minesweeper/models/cnn_residual.py:7-96), the chain conv3x3 -> GroupNorm ->
[+residual] -> ReLU -> [Dropout2d] with one kernel per layer.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import torch
from torch.utils.weak import WeakIdKeyDictionary

from . import _lib as L

COUT = 96
NGROUPS = 6
DTYPES = {torch.bfloat16: 0, torch.float16: 1}  # MC_DTYPE_BF16 / MC_DTYPE_F16 (include/mscnn.h)


def _dt(t: torch.Tensor) -> int:
    if t.dtype not in DTYPES:
        raise TypeError(f"fused kernels take bf16 or fp16 activations, got {t.dtype}")
    return DTYPES[t.dtype]


def _fn(name, argtypes):
    lib = L.load()
    f = getattr(lib, name)
    f.argtypes = argtypes
    f.restype = ctypes.c_int
    return f


_vp, _i32, _f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_float
_fwd = None


def _check(rc):
    if rc != 0:
        lib = L.load()
        lib.mc_last_error.restype = ctypes.c_char_p
        raise L.MsEnvError(lib.mc_last_error().decode(errors="replace"))


VARIANT_FWD, VARIANT_BWD, VARIANT_WGRAD = 0, 1, 2  # mc_set_variant kernels (include/msenv_debug.h)
VARIANT_TRUNK_FWD = 3  # one-launch trunk forward (<= 256 cells): 0 = default (k_trunk_fwd_pp without saves,
#   k_trunk_fwd2 with), 1 = k_trunk_fwd2 always, 2 = k_trunk_fwd_pp always


class kernel_variant:
    """Context manager: run one kernel variant (include/msenv_debug.h mc_set_variant) -- for the
    weight gradient (kernel 2) 0 = the default, 1 / 2 = k_wgrad, 3 = k_wgrad_c96; the forward and
    data backward (kernels 0 / 1) have only the per-sample kernel (0 = 1) since round 5 -- for
    parity tests of every path and same-process A/B timing."""

    def __init__(self, kernel: int, variant: int):
        self.kernel, self.variant = kernel, variant

    def __enter__(self):
        global _WGRAD_VARIANT
        _check(_fn("mc_set_variant", [_i32, _i32])(self.kernel, self.variant))
        if self.kernel == VARIANT_WGRAD:
            _WGRAD_VARIANT = self.variant
        return self

    def __exit__(self, *exc):
        global _WGRAD_VARIANT
        _check(_fn("mc_set_variant", [_i32, _i32])(self.kernel, 0))
        if self.kernel == VARIANT_WGRAD:
            _WGRAD_VARIANT = 0
        return False


_WGRAD_VARIANT = 0  # the weight-gradient variant kernel_variant set (0: the dispatcher's choice)


def prep_weight(w: torch.Tensor, cin_pad: int, dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """[96, cin, 3, 3] (f32 nn.Conv2d weight) -> ``dtype`` [9, 96, cin_pad], tap = 3*ky + kx."""
    co, ci = w.shape[0], w.shape[1]
    wt = w.permute(2, 3, 0, 1).reshape(9, co, ci)
    if cin_pad > ci:
        wt = torch.nn.functional.pad(wt, (0, cin_pad - ci))
    return wt.to(dtype).contiguous()


_enc = _c2n = None


def obs_encode(obs: torch.Tensor, codes: Optional[torch.Tensor] = None, want_nhwc: bool = False,
               cin_pad: int = 16, dtype: torch.dtype = torch.bfloat16):
    """f32 obs [N, 10, H, W] -> its cell codes (u8 [N, H, W] written into ``codes`` when
    given: 0 hidden, 1 + k revealed with k adjacent mines; exact for the env's obs) and/or,
    with ``want_nhwc``, the stem input ``dtype`` [N, H*W, cin_pad] (the planes' values cast,
    exact for any input), in one pass (mc_obs_encode). Returns the NHWC tensor or None."""
    global _enc
    if _enc is None:
        _enc = _fn("mc_obs_encode", [_vp, _vp, _vp, ctypes.c_int64, _i32, _i32, _i32, _vp])
    n, c, h, w = obs.shape
    assert c == 10 and obs.dtype == torch.float32 and obs.is_contiguous()
    if codes is not None:
        assert codes.shape == (n, h, w) and codes.dtype == torch.uint8 and codes.is_contiguous()
    x = torch.empty((n, h * w, cin_pad), dtype=dtype, device=obs.device) if want_nhwc else None
    _check(_enc(L.ptr(obs), L.ptr(codes), L.ptr(x), n, h * w, cin_pad, DTYPES[dtype], L.stream_ptr(obs.device)))
    return x


def codes_to_nhwc(codes: torch.Tensor, cin_pad: int = 16, dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """u8 cell codes [N, H, W] -> stem input ``dtype`` [N, H*W, cin_pad] (mc_codes_to_nhwc)."""
    global _c2n
    if _c2n is None:
        _c2n = _fn("mc_codes_to_nhwc", [_vp, _vp, ctypes.c_int64, _i32, _i32, _i32, _vp])
    n, h, w = codes.shape
    codes = codes.contiguous()
    x = torch.empty((n, h * w, cin_pad), dtype=dtype, device=codes.device)
    _check(_c2n(L.ptr(codes), L.ptr(x), n, h * w, cin_pad, DTYPES[dtype], L.stream_ptr(codes.device)))
    return x


def codes_to_obs(codes: torch.Tensor) -> torch.Tensor:
    """u8 cell codes [N, H, W] -> the env's f32 one-hot obs [N, 10, H, W] (exact)."""
    k = codes.long()
    planes = torch.arange(10, device=codes.device).view(1, 10, 1, 1)
    hit = (k.unsqueeze(1) == planes) | ((planes == 0) & (k.unsqueeze(1) > 0))
    return (hit & (k.unsqueeze(1) > 0)).to(torch.float32)


def obs_to_nhwc(obs: torch.Tensor, cin_pad: int = 16, dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """Stem input ``dtype`` [N, H*W, cin_pad] from an f32 obs [N, 10, H, W] (its values cast) or
    from the env's u8 cell codes [N, H, W]. One HIP pass either way."""
    if obs.dtype == torch.uint8:
        return codes_to_nhwc(obs, cin_pad, dtype)
    return obs_encode(obs.contiguous(), None, True, cin_pad, dtype)


def conv_gn_fwd(x: torch.Tensor, wt: torch.Tensor, bias: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor,
                H: int, W: int, res: Optional[torch.Tensor] = None, dmask: Optional[torch.Tensor] = None,
                save: bool = True, eps: float = 1e-5, want_mask: bool = False):
    """out = relu(GN(conv3x3(x) + bias) * gamma + beta [+ res]) [* dmask]; returns (out, y, stats),
    plus the ReLU bitmask (u8 [N, P, 12], bit j of byte c8 = out[..., 8*c8 + j] > 0) with want_mask."""
    global _fwd
    if _fwd is None:
        _fwd = _fn("mc_conv_gn_fwd", [_vp] * 11 + [_i32] * 4 + [_f32, _i32, _vp])
    n, p, cin = x.shape
    dt = _dt(x)
    assert p == H * W and x.is_contiguous()
    assert wt.shape == (9, COUT, cin) and wt.dtype == x.dtype and wt.is_contiguous()
    dev = x.device
    out = torch.empty((n, p, COUT), dtype=x.dtype, device=dev)
    y = torch.empty_like(out) if save else None
    stats = torch.empty((n, NGROUPS, 2), dtype=torch.float32, device=dev) if save else None
    rmask = torch.empty((n, p, COUT // 8), dtype=torch.uint8, device=dev) if want_mask else None
    if res is not None:
        assert res.shape == out.shape and res.dtype == x.dtype and res.is_contiguous()
    if dmask is not None:
        dmask = dmask.to(torch.float32).contiguous()
        assert dmask.shape == (n, COUT)
    f32c = lambda t: t.detach().to(torch.float32).contiguous()  # noqa: E731
    b, g, be = f32c(bias), f32c(gamma), f32c(beta)
    _check(_fwd(L.ptr(x), L.ptr(wt), L.ptr(b), L.ptr(g), L.ptr(be), L.ptr(res), L.ptr(dmask), L.ptr(out),
                L.ptr(y), L.ptr(stats), L.ptr(rmask), n, H, W, cin, eps, dt, L.stream_ptr(dev)))
    return (out, y, stats, rmask) if want_mask else (out, y, stats)


_bwd = None
_bwd_ws = None


def prep_weight_t(w: torch.Tensor, dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """[96, 96, 3, 3] nn.Conv2d weight -> ``dtype`` [9, ci, co] (the dgrad operand W[tap]^T)."""
    co, ci = w.shape[0], w.shape[1]
    return w.detach().permute(2, 3, 1, 0).reshape(9, ci, co).to(dtype).contiguous()


def dw_to_conv(dw: torch.Tensor, cin_real: int) -> torch.Tensor:
    """f32 [9, 96, cin] (tap, co, ci) -> nn.Conv2d weight layout [96, cin_real, 3, 3]."""
    return dw.view(3, 3, COUT, dw.shape[-1]).permute(2, 3, 0, 1)[:, :cin_real].contiguous()


def conv_gn_bwd(dout: torch.Tensor, out: Optional[torch.Tensor], y: torch.Tensor, stats: torch.Tensor,
                gamma: torch.Tensor, x: torch.Tensor, H: int, W: int, wT: Optional[torch.Tensor] = None,
                dmask: Optional[torch.Tensor] = None, addend: Optional[torch.Tensor] = None, want_dz: bool = False,
                rmask: Optional[torch.Tensor] = None):
    """Backward of conv_gn_fwd. Returns (dx | None, dz | None, dw f32 [9,96,cin], dgn f32 [3,96] =
    d gamma, d beta, d bias). dx (x's 16-bit type, NHWC) is produced iff the dgrad weights ``wT`` are given.
    ``rmask`` (the forward's ReLU bitmask) replaces the sign test on ``out``; one of them is needed."""
    global _bwd, _bwd_ws
    if _bwd is None:
        _bwd = _fn("mc_conv_gn_bwd", [_vp] * 16 + [ctypes.c_int64] + [_i32] * 5 + [_vp])
        _bwd_ws = _fn("mc_conv_gn_bwd_workspace", [_i32] * 4)
        _bwd_ws.restype = ctypes.c_int64
    n, p, cin = x.shape
    dev = x.device
    dt, et = _dt(x), x.dtype
    assert out is not None or rmask is not None
    for t in (dout, out, y):
        assert t is None or (t.shape == (n, p, COUT) and t.dtype == et and t.is_contiguous())
    if rmask is not None:
        assert rmask.shape == (n, p, COUT // 8) and rmask.dtype == torch.uint8 and rmask.is_contiguous()
    assert x.is_contiguous() and p == H * W
    assert stats.shape == (n, NGROUPS, 2) and stats.dtype == torch.float32
    if wT is not None:
        assert wT.shape == (9, cin, COUT) and wT.dtype == et and wT.is_contiguous()
    if addend is not None:
        assert addend.shape == (n, p, cin) and addend.dtype == et and addend.is_contiguous()
    if dmask is not None:
        dmask = dmask.to(torch.float32).contiguous()
    g = gamma.detach().to(torch.float32).contiguous()
    dy = torch.empty((n, p, COUT), dtype=et, device=dev)
    dz = torch.empty_like(dy) if want_dz else None
    dx = torch.empty((n, p, cin), dtype=et, device=dev) if wT is not None else None
    dw = torch.empty((9, COUT, cin), dtype=torch.float32, device=dev)
    dgn = torch.empty((3, COUT), dtype=torch.float32, device=dev)
    nws = int(_bwd_ws(n, H, W, cin))
    if nws < 0:
        raise L.MsEnvError("mc_conv_gn_bwd_workspace: bad sizes")
    work = torch.empty(nws, dtype=torch.float32, device=dev)
    _check(_bwd(L.ptr(dout), L.ptr(out), L.ptr(rmask), L.ptr(y), L.ptr(stats), L.ptr(g), L.ptr(dmask), L.ptr(x), L.ptr(wT),
                L.ptr(addend), L.ptr(dy), L.ptr(dz), L.ptr(dx), L.ptr(dw), L.ptr(dgn), L.ptr(work), nws,
                n, H, W, cin, dt, L.stream_ptr(dev)))
    return dx, dz, dw, dgn


# ------------------------------------------------------------------------------------
# Whole-trunk fast path for CNNResidualPolicy (cnn_residual.py:30-96): stem + residual
# blocks as fused layers, activations NHWC bf16, autograd through mc_conv_gn_bwd.

# weight -> {kind: (version, packed)}; weak keys, so a dropped model frees its packed copies
# (identity-keyed: tensor == is elementwise)
_wcache = WeakIdKeyDictionary()


def _packed(w: torch.Tensor, kind: str, dtype: torch.dtype, cin_pad: int = 0) -> torch.Tensor:
    """16-bit re-layout of a conv weight, cached until the optimizer bumps its version."""
    ent = _wcache.get(w)
    if ent is None:
        ent = _wcache[w] = {}
    hit = ent.get((kind, dtype))
    if hit is not None and hit[0] == w._version:
        return hit[1]
    t = prep_weight(w.detach(), cin_pad, dtype) if kind == "f" else prep_weight_t(w.detach(), dtype)
    ent[(kind, dtype)] = (w._version, t)
    return t


def _packed_many(ws, kind: str, dtype: torch.dtype) -> list:
    """``_packed`` of a list of 96 -> 96 conv weights: the stale ones re-laid out together, one
    stack and one permuting cast for all of them (two launches a minibatch instead of two per
    layer; the values are the per-layer re-layout's, element for element)."""
    out, stale = [None] * len(ws), []
    for i, w in enumerate(ws):
        ent = _wcache.get(w)
        hit = ent.get((kind, dtype)) if ent is not None else None
        if hit is not None and hit[0] == w._version:
            out[i] = hit[1]
        else:
            stale.append(i)
    if len(stale) == 1:
        out[stale[0]] = _packed(ws[stale[0]], kind, dtype, COUT)
    elif stale:
        src = torch.stack([ws[i].detach() for i in stale])  # [S, co, ci, 3, 3]
        assert src.shape[1:] == (COUT, COUT, 3, 3)
        dst = torch.empty((len(stale), 3, 3, COUT, COUT), dtype=dtype, device=src.device)
        dst.copy_(src.permute(0, 3, 4, 1, 2) if kind == "f" else src.permute(0, 3, 4, 2, 1))
        dst = dst.view(len(stale), 9, COUT, COUT)
        for j, i in enumerate(stale):
            ent = _wcache.get(ws[i])
            if ent is None:
                ent = _wcache[ws[i]] = {}
            out[i] = dst[j]
            ent[(kind, dtype)] = (ws[i]._version, out[i])
    return out


def trunk_layers(model) -> list:
    """[(conv, norm)] in execution order: stem, then (conv1, norm1), (conv2, norm2) per block."""
    layers = [(model.stem[0], model.stem[1])]
    for blk in model.residual_stack:
        layers += [(blk.conv1, blk.norm1), (blk.conv2, blk.norm2)]
    return layers


# ------------------------------------------------------------------------------------
# The residual stack in one launch per direction (csrc/mscnn_trunk.hip, include/mscnn.h
# mc_trunk_fwd / mc_trunk_bwd): bitwise the per-layer path, without the per-layer HBM round
# trips of the activations. ``CHAIN`` selects it (the default);
# ``chain_path(False)`` runs the per-layer kernels, for parity tests and A/B timing.

CHAIN = os.environ.get("MS_TRUNK_CHAIN", "1") != "0"  # MS_TRUNK_CHAIN=0: per-layer kernels (A/B runs)
MAX_CHAIN_LAYERS = 16  # MC_TRUNK_MAX_LAYERS


class chain_path:
    """Context manager: run the trunk through the one-launch kernels (True) or per layer (False)."""

    def __init__(self, on: bool):
        self.on = on

    def __enter__(self):
        global CHAIN
        self.prev, CHAIN = CHAIN, self.on
        return self

    def __exit__(self, *exc):
        global CHAIN
        CHAIN = self.prev
        return False


class _FwdLayer(ctypes.Structure):  # mc_fwd_layer
    _fields_ = [(n, _vp) for n in ("w", "bias", "gamma", "beta", "dmask", "out", "ysave", "stats", "relu_mask")]


class _BwdLayer(ctypes.Structure):  # mc_bwd_layer
    _fields_ = [(n, _vp) for n in ("ysave", "stats", "gamma", "relu_mask", "dmask", "wT", "dy")]


_tf = _tfws = _tb = _tbws = _wg = _wgn = None


def _trunk_bind():
    global _tf, _tfws, _tb, _tbws, _wg, _wgn
    if _tf is None:
        _tf = _fn("mc_trunk_fwd_pooled", [_vp, ctypes.POINTER(_FwdLayer), _i32, _vp, ctypes.c_int64, _vp]
                  + [_i32] * 3 + [_f32, _i32, _vp])
        _tfws = _fn("mc_trunk_fwd_workspace", [_i32] * 3)
        _tfws.restype = ctypes.c_int64
        _tb = _fn("mc_trunk_bwd", [_vp, ctypes.POINTER(_BwdLayer), _i32, _vp, _vp, ctypes.c_int64] + [_i32] * 4
                  + [_vp])
        _tbws = _fn("mc_trunk_bwd_workspace", [_i32] * 4)
        _tbws.restype = ctypes.c_int64
        _wg = _fn("mc_conv_wgrad", [_vp] * 4 + [ctypes.c_int64] + [_i32] * 5 + [_vp])
        _wgn = _fn("mc_conv_wgrad_gn", [_vp] * 8 + [ctypes.c_int64] + [_i32] * 4 + [_vp])


def chain_ok(layers, H: int, W: int) -> bool:
    """The one-launch trunk takes 96-channel residual stacks of at most 8 blocks on boards of
    at most 512 cells (the per-layer kernels' range)."""
    nres = len(layers) - 1
    return CHAIN and 0 < nres <= MAX_CHAIN_LAYERS and nres % 2 == 0 and H * W <= 512 and W <= 64


WGRAD_GN = True  # False: the forward writes every conv1 output and mc_conv_wgrad reads it (A/B timing)


def wgrad_gn_ok(H: int, W: int) -> bool:
    """mc_conv_wgrad_gn's range: 16x16 boards under the default (or c96) weight gradient."""
    return WGRAD_GN and H == 16 and W == 16 and _WGRAD_VARIANT in (0, 3)


def trunk_forward_chain(x, layers, H: int, W: int, dmasks, save: bool, pooled: Optional[torch.Tensor] = None):
    """Residual stack (layers[1:]) on the stem output ``x`` [N, P, 96] in one mc_trunk_fwd.
    Returns (out, outs, ys, sts, rms): per layer lists of the saved tensors (empty unless ``save``).
    Where mc_conv_wgrad_gn applies (``wgrad_gn_ok``), a block's conv1 output is not written: its
    entry in ``outs`` is None and the backward recomputes it from the layer's y inside the weight
    gradient. ``pooled`` (f32 [N, 96]) receives the output's mean over the pixels."""
    _trunk_bind()
    n, p, c = x.shape
    assert c == COUT and x.is_contiguous() and p == H * W
    dev, et = x.device, x.dtype
    res = layers[1:]
    nl = len(res)
    arr = (_FwdLayer * nl)()
    keep = []  # f32 parameter copies must outlive the enqueue (the allocator may reuse their memory only after)
    outs, ys, sts, rms = [], [], [], []
    eps = res[0][1].eps
    wts = _packed_many([conv.weight for conv, _ in res], "f", et)
    for k, (conv, norm) in enumerate(res):
        assert norm.eps == eps and conv.weight.shape[0] == COUT and conv.weight.shape[1] == COUT
        f32c = lambda t: t.detach().to(torch.float32).contiguous()  # noqa: E731
        b, g, be = f32c(conv.bias), f32c(norm.weight), f32c(norm.bias)
        dm = None
        if k % 2 == 0 and dmasks is not None:  # conv1 of block k // 2: Dropout2d after its ReLU
            dm = dmasks[k // 2].to(torch.float32).contiguous()
            assert dm.shape == (n, COUT)
        last = k == nl - 1
        keep_out = save and not (k % 2 == 0 and wgrad_gn_ok(H, W))
        out = torch.empty((n, p, COUT), dtype=et, device=dev) if (keep_out or last) else None
        y = torch.empty((n, p, COUT), dtype=et, device=dev) if save else None
        st = torch.empty((n, NGROUPS, 2), dtype=torch.float32, device=dev) if save else None
        rm = torch.empty((n, p, COUT // 8), dtype=torch.uint8, device=dev) if save else None
        keep += [b, g, be, dm]
        if save:
            outs.append(out)
            ys.append(y)
            sts.append(st)
            rms.append(rm)
        arr[k] = _FwdLayer(L.ptr(wts[k]), L.ptr(b), L.ptr(g), L.ptr(be), L.ptr(dm),
                           L.ptr(out), L.ptr(y), L.ptr(st), L.ptr(rm))
        if last:
            final = out
    nws = int(_tfws(n, H, W))
    work = None if save else torch.empty(max(nws, 0), dtype=torch.uint8, device=dev)
    if pooled is not None:
        assert pooled.shape == (n, COUT) and pooled.dtype == torch.float32 and pooled.is_contiguous()
    _check(_tf(L.ptr(x), arr, nl, L.ptr(work), 0 if work is None else work.numel(), L.ptr(pooled), n, H, W, eps,
               _dt(x), L.stream_ptr(dev)))
    return final, outs, ys, sts, rms


def trunk_backward_chain(dout, layers, ys, sts, rms, dmasks, H: int, W: int):
    """GroupNorm + data backward of the stem (layers[0]) and the residual stack in one
    mc_trunk_bwd. Returns (dys, dgn): per layer dL/dy [N, P, 96] and d gamma / d beta / d bias f32
    [nlayers, 3, 96]."""
    _trunk_bind()
    n, p, _ = dout.shape
    dev, et = dout.device, dout.dtype
    nl = len(layers)
    arr = (_BwdLayer * nl)()
    keep, dys = [], []
    wTs = [None] + _packed_many([conv.weight for conv, _ in layers[1:]], "t", et)
    for li, (conv, norm) in enumerate(layers):
        g = norm.weight.detach().to(torch.float32).contiguous()
        dm = None
        if li % 2 == 1 and dmasks is not None:
            dm = dmasks[(li - 1) // 2].to(torch.float32).contiguous()
        wT = wTs[li]
        dy = torch.empty((n, p, COUT), dtype=et, device=dev)
        keep += [g, dm]
        dys.append(dy)
        arr[li] = _BwdLayer(L.ptr(ys[li]), L.ptr(sts[li]), L.ptr(g), L.ptr(rms[li]), L.ptr(dm), L.ptr(wT), L.ptr(dy))
    dgn = torch.empty((nl, 3, COUT), dtype=torch.float32, device=dev)
    nws = int(_tbws(nl, n, H, W))
    if nws < 0:
        raise L.MsEnvError("mc_trunk_bwd_workspace: bad sizes")
    work = torch.empty(nws, dtype=torch.uint8, device=dev)
    _check(_tb(L.ptr(dout), arr, nl, L.ptr(dgn), L.ptr(work), nws, n, H, W, _dt(dout), L.stream_ptr(dev)))
    return dys, dgn


def conv_wgrad_gn(dy: torch.Tensor, y: torch.Tensor, stats: torch.Tensor, norm, dmask: Optional[torch.Tensor],
                  H: int, W: int) -> torch.Tensor:
    """conv_wgrad with x = the GroupNorm + ReLU (+ Dropout2d) output of the layer that saved ``y`` /
    ``stats`` (``norm`` its GroupNorm, ``dmask`` [N, 96] or None), recomputed in the kernel
    (mc_conv_wgrad_gn): bitwise conv_wgrad on the forward's x."""
    _trunk_bind()
    global _bwd_ws
    if _bwd_ws is None:
        _bwd_ws = _fn("mc_conv_gn_bwd_workspace", [_i32] * 4)
        _bwd_ws.restype = ctypes.c_int64
    n, p, c = y.shape
    assert c == COUT and dy.shape == y.shape and dy.dtype == y.dtype and y.is_contiguous() and dy.is_contiguous()
    g = norm.weight.detach().to(torch.float32).contiguous()
    b = norm.bias.detach().to(torch.float32).contiguous()
    dm = dmask.to(torch.float32).contiguous() if dmask is not None else None
    dw = torch.empty((9, COUT, COUT), dtype=torch.float32, device=y.device)
    nws = int(_bwd_ws(n, H, W, COUT))
    work = torch.empty(nws, dtype=torch.float32, device=y.device)
    _check(_wgn(L.ptr(dy), L.ptr(y), L.ptr(stats), L.ptr(g), L.ptr(b), L.ptr(dm), L.ptr(dw), L.ptr(work), nws, n, H, W,
                _dt(y), L.stream_ptr(y.device)))
    return dw


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """Weight gradient f32 [9, 96, cin] (tap, co, ci) of a conv3x3 layer from dL/dy and its input
    (mc_conv_wgrad; mc_conv_gn_bwd's second half)."""
    _trunk_bind()
    global _bwd_ws
    if _bwd_ws is None:
        _bwd_ws = _fn("mc_conv_gn_bwd_workspace", [_i32] * 4)
        _bwd_ws.restype = ctypes.c_int64
    n, p, cin = x.shape
    assert dy.shape == (n, p, COUT) and dy.dtype == x.dtype and x.is_contiguous() and dy.is_contiguous()
    dw = torch.empty((9, COUT, cin), dtype=torch.float32, device=x.device)
    nws = int(_bwd_ws(n, H, W, cin))
    work = torch.empty(nws, dtype=torch.float32, device=x.device)
    _check(_wg(L.ptr(dy), L.ptr(x), L.ptr(dw), L.ptr(work), nws, n, H, W, cin, _dt(x), L.stream_ptr(x.device)))
    return dw


def _trunk_forward(x0, layers, H, W, dmasks, save, pooled=None):
    """Runs every layer; with ``save`` returns the tensors the backward needs:
    acts[l] = input of layer l (acts[l + 1] = its output), ys[l], sts[l], and the ReLU bitmasks.
    ``pooled`` (f32 [N, 96]): receives the output's mean over the pixels."""
    if not chain_ok(layers, H, W):
        x, acts, ys, sts, rms = _trunk_forward_layers(x0, layers, H, W, dmasks, save)
        if pooled is not None:
            pooled.copy_(x.mean(1, dtype=torch.float32))
        return x, acts, ys, sts, rms
    conv, norm = layers[0]
    wt = _packed(conv.weight, "f", x0.dtype, x0.shape[-1])
    if save:
        x, y, st, rm = conv_gn_fwd(x0, wt, conv.bias, norm.weight, norm.bias, H, W, save=True, eps=norm.eps,
                                   want_mask=True)
    else:
        x, _, _ = conv_gn_fwd(x0, wt, conv.bias, norm.weight, norm.bias, H, W, save=False, eps=norm.eps)
    out, outs, ys, sts, rms = trunk_forward_chain(x, layers, H, W, dmasks, save, pooled=pooled)
    if not save:
        return out, [], [], [], []
    return out, [x0, x] + outs, [y] + ys, [st] + sts, [rm] + rms


def _trunk_forward_layers(x0, layers, H, W, dmasks, save):
    """_trunk_forward through the per-layer kernels."""
    acts, ys, sts, rms = [x0], [], [], []
    x, blk_in = x0, None
    for li, (conv, norm) in enumerate(layers):
        wt = _packed(conv.weight, "f", x.dtype, x.shape[-1])
        res = dm = None
        if li % 2 == 1:  # first half of a block: Dropout2d after the ReLU
            blk_in = x
            dm = dmasks[(li - 1) // 2] if dmasks is not None else None
        elif li > 0:  # second half: + the block input, then ReLU
            res = blk_in
        if save:
            x, y, st, rm = conv_gn_fwd(x, wt, conv.bias, norm.weight, norm.bias, H, W, res=res, dmask=dm,
                                       save=True, eps=norm.eps, want_mask=True)
            acts.append(x)
            ys.append(y)
            sts.append(st)
            rms.append(rm)
        else:
            x, _, _ = conv_gn_fwd(x, wt, conv.bias, norm.weight, norm.bias, H, W, res=res, dmask=dm,
                                  save=False, eps=norm.eps)
    return x, acts, ys, sts, rms


class _TrunkFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x0, H, W, dmasks, layers, *params):
        """-> (features, pooled): pooled = the features' f32 mean over the pixels, an output
        without a gradient of its own (the heads' backward adds its gradient to df)."""
        ctx.chain = chain_ok(layers, H, W)  # the backward takes the path the forward took
        pooled = torch.empty((x0.shape[0], COUT), dtype=torch.float32, device=x0.device)
        out, acts, ys, sts, rms = _trunk_forward(x0, layers, H, W, dmasks, save=True, pooled=pooled)
        ctx.H, ctx.W, ctx.layers, ctx.dmasks = H, W, layers, dmasks
        ctx.saved = (acts, ys, sts, rms)
        ctx.nparams = len(params)
        ctx.mark_non_differentiable(pooled)
        return out, pooled

    @staticmethod
    def backward(ctx, dout, _dpooled):
        acts, ys, sts, rms = ctx.saved
        layers, H, W, dmasks = ctx.layers, ctx.H, ctx.W, ctx.dmasks
        grads = {}
        d = dout.to(acts[0].dtype).contiguous()
        nl = len(layers)
        if ctx.chain:
            dys, dgn = trunk_backward_chain(d, layers, ys, sts, rms, dmasks, H, W)
            ctx.saved = None
            out = [None, None, None, None, None]
            for li, (conv, norm) in enumerate(layers):
                if acts[li] is None:  # a block's conv1 output, not written by the forward
                    dm = dmasks[(li - 2) // 2] if dmasks is not None else None
                    dw = conv_wgrad_gn(dys[li], ys[li - 1], sts[li - 1], layers[li - 1][1], dm, H, W)
                else:
                    dw = conv_wgrad(dys[li], acts[li], H, W)
                dys[li] = None
                gs = (dw_to_conv(dw, conv.weight.shape[1]), dgn[li, 2], dgn[li, 0], dgn[li, 1])
                for p, g in zip((conv.weight, conv.bias, norm.weight, norm.bias), gs):
                    out.append(g.to(p.dtype) if p.requires_grad else None)
            return tuple(out)
        skip = None  # dz of a block's second half: the block input's skip gradient
        for li in range(nl - 1, -1, -1):
            conv, norm = layers[li]
            x = acts[li]
            cin_real = conv.weight.shape[1]
            want_dx = li > 0
            dm = dmasks[(li - 1) // 2] if (dmasks is not None and li % 2 == 1) else None
            addend = skip if li % 2 == 1 else None
            dx, dz, dw, dgn = conv_gn_bwd(d, None, ys[li], sts[li], norm.weight, x, H, W,
                                          wT=_packed(conv.weight, "t", x.dtype) if want_dx else None, dmask=dm,
                                          addend=addend, want_dz=(li % 2 == 0 and li > 0), rmask=rms[li])
            skip = dz
            grads[id(conv.weight)] = dw_to_conv(dw, cin_real)
            grads[id(conv.bias)] = dgn[2]
            grads[id(norm.weight)] = dgn[0]
            grads[id(norm.bias)] = dgn[1]
            d = dx
        ctx.saved = None
        out = [None, None, None, None, None]
        for conv, norm in layers:
            for p in (conv.weight, conv.bias, norm.weight, norm.bias):
                g = grads[id(p)]
                out.append(g.to(p.dtype) if p.requires_grad else None)
        return tuple(out)


def trunk_params(layers) -> list:
    return [p for conv, norm in layers for p in (conv.weight, conv.bias, norm.weight, norm.bias)]


def fused_features(model, obs: torch.Tensor, dtype: torch.dtype = torch.bfloat16,
                   dmasks: Optional[list] = None, with_pooled: bool = False):
    """Trunk features of CNNResidualPolicy as NHWC ``dtype`` [N, H*W, 96] via the fused kernels
    (``dtype``: the autocast type, bf16 or fp16). ``dmasks``: per-block Dropout2d masks [N, 96]
    (keep / (1 - p), ms_amd.dropout); without them a training-mode model draws torch-RNG masks.
    ``with_pooled``: returns (features, their f32 mean over the pixels [N, 96]), the mean taken by
    the trunk kernel from the last tile on chip (no gradient of its own: heads_apply routes the
    value head's gradient into df)."""
    n, H, W = obs.shape[0], obs.shape[-2], obs.shape[-1]  # f32 obs [N, 10, H, W] or u8 codes [N, H, W]
    layers = trunk_layers(model)
    x0 = obs_to_nhwc(obs, 16, dtype)
    nblk = len(model.residual_stack)
    p = model.dropout_p()
    if dmasks is None and model.training and p > 0:
        keep = torch.rand(nblk, n, COUT, device=obs.device) >= p
        dmasks = [(keep[i].float() * (1.0 / (1.0 - p))).contiguous() for i in range(nblk)]
    elif not (model.training and p > 0):
        dmasks = None
    params = trunk_params(layers)
    if torch.is_grad_enabled() and any(q.requires_grad for q in params):
        out, pooled = _TrunkFn.apply(x0, H, W, dmasks, layers, *params)
        return (out, pooled) if with_pooled else out
    pooled = torch.empty((n, COUT), dtype=torch.float32, device=obs.device) if with_pooled else None
    out, _, _, _, _ = _trunk_forward(x0, layers, H, W, dmasks, save=False, pooled=pooled)
    return (out, pooled) if with_pooled else out


# ------------------------------------------------------------------------------------
# Policy / belief heads + the value head's global average pool on NHWC features
# (cnn_residual.py:57-96) through csrc/msheads.hip.

_hf = _hb = _hbws = None
_hcache: dict = {}


def _head_pack(pol, mine, dtype: torch.dtype):
    """``dtype`` [192|96, 96] W1 (policy rows first), its policy transpose, f32 b1 / w2 / b2."""
    heads = [pol] + ([mine] if mine is not None else [])
    params = tuple(t for h in heads for m in (h[0], h[2]) for t in (m.weight, m.bias))
    vers = tuple(t._version for t in params)
    # the entry holds the parameters themselves and compares by identity: ids of freed
    # parameters can be reused by a new model at the same versions
    key = (len(heads), dtype)
    hit = _hcache.get(key)
    if hit is not None and hit[1] == vers and all(a is b for a, b in zip(hit[0], params)):
        return hit[2]
    w1 = torch.cat([h[0].weight.detach().reshape(COUT, COUT) for h in heads]).to(dtype).contiguous()
    b1 = torch.cat([h[0].bias.detach() for h in heads]).float().contiguous()
    w2 = torch.cat([h[2].weight.detach().reshape(COUT) for h in heads]).float().contiguous()
    b2 = torch.cat([h[2].bias.detach().reshape(1) for h in heads]).float().contiguous()
    packed = (w1, b1, w2, b2)
    _hcache[key] = (params, vers, packed)
    return packed


def _heads_bind():
    global _hf, _hb, _hbws
    if _hf is None:
        _hf = _fn("mc_heads_fwd", [_vp] * 7 + [ctypes.c_int64, _i32, _vp])
        _hb = _fn("mc_heads_bwd", [_vp] * 8 + [_i32] + [_vp] * 5 + [ctypes.c_int64, ctypes.c_int64, _i32, _vp])
        _hbws = _fn("mc_heads_bwd_workspace", [ctypes.c_int64])
        _hbws.restype = ctypes.c_int64


def heads_forward(f: torch.Tensor, pol, mine=None):
    """f bf16 | fp16 [N, P, 96] -> policy logits f32 [N, P] (and mine logits f32 [N, P] when ``mine``)."""
    _heads_bind()
    n, p, c = f.shape
    dt = _dt(f)
    assert c == COUT and f.is_contiguous()
    w1, b1, w2, b2 = _head_pack(pol, mine, f.dtype)
    lp = torch.empty((n, p), dtype=torch.float32, device=f.device)
    lm = torch.empty_like(lp) if mine is not None else None
    _check(_hf(L.ptr(f), L.ptr(w1), L.ptr(b1), L.ptr(w2), L.ptr(b2), L.ptr(lp), L.ptr(lm), n * p, dt,
               L.stream_ptr(f.device)))
    return lp, lm


class _HeadsFn(torch.autograd.Function):
    """(f, head params) -> (policy logits, pooled features, mine logits). The mine head
    reads f.detach() (cnn_residual.py:94), so its gradient never reaches f."""

    @staticmethod
    def forward(ctx, f, pol, mine, pre, *params):
        lp, lm = heads_forward(f, pol, mine)
        # the trunk kernel's mean (``pre``), or f32 accumulation here (no f32 copy of f)
        pooled = pre.clone() if pre is not None else f.mean(1, dtype=torch.float32)
        ctx.save_for_backward(f)
        ctx.pol, ctx.mine = pol, mine
        return lp, pooled, lm

    @staticmethod
    def backward(ctx, dlp, dpool, dlm):
        (f,) = ctx.saved_tensors
        pol, mine = ctx.pol, ctx.mine
        _heads_bind()
        n, p, _ = f.shape
        M = n * p
        # the kernel always runs both heads' math; without a mine head its rows get dl = 0
        w1, b1, w2, _ = _head_pack(pol, mine if mine is not None else pol, f.dtype)
        dev = f.device
        dlp = dlp.float().contiguous() if dlp is not None else torch.zeros(n, p, device=dev)
        dlm = dlm.float().contiguous() if (dlm is not None and mine is not None) else None
        gadd = (dpool.float() / p).contiguous() if dpool is not None else None
        df = torch.empty_like(f)
        dw1 = torch.empty(2 * COUT, COUT, device=dev)
        db1 = torch.empty(2 * COUT, device=dev)
        dw2 = torch.empty(2 * COUT, device=dev)
        nws = int(_hbws(M))
        work = torch.empty(nws, device=dev)
        _check(_hb(L.ptr(f), L.ptr(dlp), L.ptr(dlm), L.ptr(w1), None, L.ptr(b1), L.ptr(w2), L.ptr(gadd), p,
                   L.ptr(df), L.ptr(dw1), L.ptr(db1), L.ptr(dw2), L.ptr(work), nws, M, _dt(f), L.stream_ptr(dev)))
        grads = [df, None, None, None]
        for h, i, dl in [(pol, 0, dlp)] + ([(mine, 1, dlm)] if mine is not None else []):
            sl = slice(i * COUT, (i + 1) * COUT)
            db2 = dl.sum() if dl is not None else torch.zeros((), device=dev)
            grads += [dw1[sl].reshape(h[0].weight.shape), db1[sl], dw2[sl].reshape(h[2].weight.shape),
                      db2.reshape(h[2].bias.shape)]
        return tuple(grads)


def heads_apply(f: torch.Tensor, pol, mine=None, pooled: Optional[torch.Tensor] = None):
    """Policy logits f32 [N, P], pooled trunk features f32 [N, 96], mine logits [N, P] | None.
    ``pooled``: f's mean over the pixels when the trunk already took it (fused_features)."""
    params = []
    for h in [pol] + ([mine] if mine is not None else []):
        params += [h[0].weight, h[0].bias, h[2].weight, h[2].bias]
    if torch.is_grad_enabled() and (f.requires_grad or any(q.requires_grad for q in params)):
        return _HeadsFn.apply(f, pol, mine, pooled, *params)
    lp, lm = heads_forward(f, pol, mine)
    return lp, (pooled if pooled is not None else f.mean(1, dtype=torch.float32)), lm


# ------------------------------------------------------------------------------------
# The value head's MLP (cnn_residual.py:64-72: Linear 96 -> H, ReLU, Linear H -> H, ReLU,
# Linear H -> 1) on the pooled features under 16-bit autocast.

VALUE_SPLITK = 32  # row chunks of the weight gradients' batched GEMMs; 0: autocast's nn.Linear chain


class _ValueMLP(torch.autograd.Function):
    """Forward exactly as autocast runs the three nn.Linear (16-bit addmm with 16-bit bias, ReLU
    in 16 bits). Backward: the data gradients as autocast's (16-bit GEMMs), the weight gradients
    as f32 split-K batched GEMMs over row chunks plus a fixed-order sum -- hipBLASLt runs the
    K = N (32,768 rows) weight-gradient GEMMs at ~115 us each (tools/vhead_micro.py: 0.39 vs
    0.55-0.63 ms a minibatch); they are f32 sums of the same 16-bit products, so they differ from
    autocast's 16-bit-rounded weight gradients by at most that rounding."""

    @staticmethod
    def forward(ctx, pooled, dt, w1, b1, w2, b2, w3, b3):
        x = pooled.to(dt)
        W = [w.detach().to(dt) for w in (w1, w2, w3)]
        a1 = torch.addmm(b1.detach().to(dt), x, W[0].t())
        h1 = torch.relu(a1)
        a2 = torch.addmm(b2.detach().to(dt), h1, W[1].t())
        h2 = torch.relu(a2)
        v = torch.addmm(b3.detach().to(dt), h2, W[2].t())
        ctx.save_for_backward(x, h1, h2, *W)
        return v

    @staticmethod
    def backward(ctx, dv):
        x, h1, h2, W1, W2, W3 = ctx.saved_tensors
        dv = dv.to(x.dtype)
        n = x.shape[0]
        s = VALUE_SPLITK if n % VALUE_SPLITK == 0 and n >= 64 * VALUE_SPLITK else 1

        def wgrad(d, a):  # d^T a in f32, summed over s row chunks in order
            d32, a32 = d.float(), a.float()
            if s == 1:
                return d32.t() @ a32
            return torch.bmm(d32.view(s, n // s, -1).transpose(1, 2), a32.view(s, n // s, -1)).sum(0)

        dh2 = (dv @ W3) * (h2 > 0)
        dh1 = (dh2 @ W2) * (h1 > 0)
        dx = (dh1 @ W1).float()
        return (dx, None, wgrad(dh1, x), dh1.float().sum(0), wgrad(dh2, h1), dh2.float().sum(0),
                wgrad(dv, h2), dv.float().sum(0))


def value_mlp(vh, pooled: torch.Tensor) -> torch.Tensor:
    """value [N] of the value head ``vh`` (nn.Sequential pool, flatten, Linear, ReLU, Linear,
    ReLU, Linear) on ``pooled`` f32 [N, 96], under the active 16-bit autocast."""
    l1, l2, l3 = vh[2], vh[4], vh[6]
    dt = torch.get_autocast_dtype("cuda")
    params = (l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias)
    if VALUE_SPLITK and torch.is_grad_enabled() and (pooled.requires_grad or any(p.requires_grad for p in params)):
        return _ValueMLP.apply(pooled, dt, *params).squeeze(-1)
    return l3(torch.relu(l2(torch.relu(l1(pooled))))).squeeze(-1)

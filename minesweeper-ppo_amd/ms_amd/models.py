"""Policy/value/belief networks, state_dict-compatible with the reference.

Reference: minesweeper/models/cnn_residual.py:7-99 (CNNResidualPolicy),
minesweeper/models/cnn.py:7-60 (CNNPolicy), minesweeper/models/__init__.py:17-49
(build_model). Module attribute names, Sequential indices and parameter
creation order are the reference's, so (a) checkpoints load unchanged
(``stem.{0,1}``, ``residual_stack.{i}.{conv1,norm1,conv2,norm2}``,
``policy_head.{0,2}``, ``value_head.{2,4,6}``, ``mine_head.{0,2}``) and
(b) ``torch.manual_seed(s)`` yields bit-identical initial weights (checked
against tests/golden/model_full_*.npz).

MI355X notes: on a HIP device under bf16 or fp16 autocast with the shipped trunk
width (96), the residual trunk and the policy / belief heads run as hand-written
MFMA kernels (csrc/mscnn*.hip, csrc/msheads.hip via ms_amd.fused).
Every other case (fp32, CPU, other widths) runs the PyTorch op chain below;
``model.fused = False`` forces that chain. Dropout2d masks come from the keyed
hash of ms_amd.dropout when a key is set (the Trainer sets one per forward), so a
data-parallel rank draws the masks its samples get in a one-GPU run.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import exact_fp32_convs


class GroupNorm(nn.GroupNorm):
    """nn.GroupNorm with the affine step done as plain elementwise ops.

    Same parameters / state_dict as nn.GroupNorm. On this image's PyTorch-ROCm
    (2.10 + ROCm 7.0, gfx950) the fused GroupNorm backward returns wrong
    weight/bias gradients once the batch reaches 256 samples (input gradients
    stay right; tools/gn_torch_check.py), and PPO minibatches are
    far above that. Normalising without affine and applying gamma/beta
    elementwise keeps autograd on correct kernels."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:  # CPU kernels are right: keep the reference's exact op
            return super().forward(x)
        y = F.group_norm(x, self.num_groups, None, None, self.eps)
        if not self.affine:
            return y
        shape = (1, -1) + (1,) * (x.dim() - 2)
        return y * self.weight.view(shape) + self.bias.view(shape)


def _conv3(cin: int, cout: int) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=3, padding=1)


def _pointwise_head(channels: int) -> nn.Sequential:
    """1x1 conv -> ReLU -> 1x1 conv to one map (policy_head / mine_head layout)."""
    return nn.Sequential(nn.Conv2d(channels, channels, kernel_size=1), nn.ReLU(inplace=True),
                         nn.Conv2d(channels, 1, kernel_size=1))


class _ResidualBlock(nn.Module):
    """conv3x3-GN-ReLU-Dropout2d-conv3x3-GN, + skip, ReLU (cnn_residual.py:7-27)."""

    def __init__(self, channels: int, groups: int, dropout: float = 0.0) -> None:
        super().__init__()
        self.conv1 = _conv3(channels, channels)
        self.norm1 = GroupNorm(groups, channels)
        self.conv2 = _conv3(channels, channels)
        self.norm2 = GroupNorm(groups, channels)
        self.dropout = nn.Dropout2d(dropout) if dropout > 0 else nn.Identity()
        self.act = nn.ReLU(inplace=True)

    def forward(self, x: torch.Tensor, dmask: Optional[torch.Tensor] = None) -> torch.Tensor:
        y = self.act(self.norm1(self.conv1(x)))
        # dmask: keyed Dropout2d mask [N, C] (keep / (1 - p)), in place of the torch-RNG draw
        # (y is f32 here: group_norm is on autocast's fp32 list, so this is nn.Dropout2d's f32
        # product; for a 16-bit y ATen would round the 1/(1-p) scale to y's dtype first)
        y = (y.float() * dmask.float()[:, :, None, None]).to(y.dtype) if dmask is not None else self.dropout(y)
        y = self.norm2(self.conv2(y))
        return self.act(y + x)


class CNNResidualPolicy(nn.Module):
    """Residual CNN trunk + policy (per-cell logit), value (GAP MLP) and
    detached belief (per-cell mine logit) heads (cnn_residual.py:30-99)."""

    def __init__(self, in_channels: int, *, stem_channels: int = 128, blocks: int = 6,
                 dropout: float = 0.05, value_hidden: int = 256) -> None:
        super().__init__()
        exact_fp32_convs()  # fp32 3x3 convolutions without MIOpen's Winograd (ms_amd.exact_fp32_convs)
        if stem_channels <= 0:
            raise ValueError("stem_channels must be positive")
        if blocks <= 0:
            raise ValueError("blocks must be positive")
        C = stem_channels
        groups = max(1, C // 16)
        self.stem = nn.Sequential(_conv3(in_channels, C), GroupNorm(groups, C), nn.ReLU(inplace=True))
        self.residual_stack = nn.Sequential(*(_ResidualBlock(C, groups, dropout) for _ in range(blocks)))
        self.policy_head = _pointwise_head(C)
        self.value_head = nn.Sequential(
            nn.AdaptiveAvgPool2d(1), nn.Flatten(),
            nn.Linear(C, value_hidden), nn.ReLU(inplace=True),
            nn.Linear(value_hidden, value_hidden), nn.ReLU(inplace=True),
            nn.Linear(value_hidden, 1),
        )
        self.mine_head = _pointwise_head(C)

        # fused MFMA trunk + heads (csrc/mscnn*.hip, csrc/msheads.hip) on HIP devices under
        # bf16 or fp16 autocast; False forces the PyTorch op chain
        self.fused = True
        self._dropout_key = None  # (global sample ids, seed, counter): ms_amd.dropout.keyed_dropout

    def set_gradient_checkpointing(self, enabled: bool) -> None:  # API parity (no-op, as the reference)
        return None

    def use_fused(self, x: torch.Tensor) -> bool:
        conv0 = self.stem[0]
        return (self.fused and x.is_cuda and conv0.out_channels == 96 and conv0.in_channels <= 16
                and x.shape[-2] * x.shape[-1] <= 512 and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") in (torch.bfloat16, torch.float16))

    def dropout_p(self) -> float:
        d = self.residual_stack[0].dropout
        return float(d.p) if isinstance(d, nn.Dropout2d) else 0.0

    def keyed_masks(self, n: int) -> Optional[list]:
        """Per-block Dropout2d masks [N, C] from the keyed hash, when a key is set, the model
        is training and dropout is on; None otherwise (torch-RNG Dropout2d applies)."""
        key = self._dropout_key
        p = self.dropout_p()
        if key is None or not self.training or p <= 0:
            return None
        rows, seed, counter = key
        if rows.shape[0] != n:
            raise ValueError(f"dropout key holds {rows.shape[0]} sample ids for a batch of {n}")
        from .dropout import dropout_masks
        m = dropout_masks(rows, len(self.residual_stack), self.stem[0].out_channels, p, seed, counter)
        return list(m.unbind(0))

    def features(self, x: torch.Tensor, dmasks: Optional[list] = None) -> torch.Tensor:
        f = self.stem(x)
        for i, blk in enumerate(self.residual_stack):
            f = blk(f, dmasks[i] if dmasks is not None else None)
        return f

    def _heads_fused(self, f: torch.Tensor, H: int, W: int, return_mine: bool, pooled=None):
        """Heads through csrc/msheads.hip: policy + mine logits in one pass over f; the pooled
        features come from the trunk kernel (``pooled``); the value MLP (N x 96 -> 1) is
        PyTorch GEMMs with split-K weight gradients (fused.value_mlp)."""
        from .fused import heads_apply, value_mlp
        logits, pooled, mine = heads_apply(f, self.policy_head, self.mine_head if return_mine else None, pooled)
        value = value_mlp(self.value_head, pooled)
        if return_mine:
            return logits, value, mine.view(f.shape[0], 1, H, W)
        return logits, value

    def forward(self, x: torch.Tensor, return_mine: bool = False):
        """x: the env's f32 obs [N, 10, H, W], or its u8 cell codes [N, H, W] (the Trainer's
        rollout-buffer layout, ms_amd.fused.obs_encode)."""
        dmasks = self.keyed_masks(x.shape[0])
        if self.use_fused(x):
            from .fused import fused_features
            f, pooled = fused_features(self, x, torch.get_autocast_dtype("cuda"), dmasks=dmasks, with_pooled=True)
            return self._heads_fused(f, x.shape[-2], x.shape[-1], return_mine, pooled)
        if x.dtype == torch.uint8:
            from .fused import codes_to_obs
            x = codes_to_obs(x)
        f = self.features(x, dmasks)
        n = f.shape[0]
        # [N,1,H,W] -> [N,H*W], index r*W + c (cnn_residual.py:89)
        logits = self.policy_head(f).reshape(n, -1)
        value = self.value_head(f).squeeze(-1)
        if return_mine:
            return logits, value, self.mine_head(f.detach())
        return logits, value

    def beta_regularizer(self) -> torch.Tensor:
        return next(self.parameters()).new_zeros(())


class CNNPolicy(nn.Module):
    """Three-conv baseline (cnn.py:7-60); the trainer's default when the YAML
    names no model (train_rl.py:369)."""

    def __init__(self, in_channels: int, hidden: int = 64) -> None:
        super().__init__()
        exact_fp32_convs()  # fp32 3x3 convolutions without MIOpen's Winograd (ms_amd.exact_fp32_convs)
        hidden = int(hidden)
        if hidden <= 0:
            raise ValueError("hidden must be positive")
        feat = 64
        self.backbone = nn.Sequential(
            _conv3(in_channels, 32), nn.ReLU(inplace=True), GroupNorm(4, 32),
            _conv3(32, 64), nn.ReLU(inplace=True), GroupNorm(8, 64),
            _conv3(64, feat), nn.ReLU(inplace=True),
        )
        self.policy_head = nn.Conv2d(feat, 1, kernel_size=1)
        self.value_head = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(feat, hidden),
                                        nn.ReLU(inplace=True), nn.Linear(hidden, 1))
        self.mine_head = nn.Conv2d(feat, 1, kernel_size=1)

    def set_gradient_checkpointing(self, enabled: bool) -> None:
        return None

    def forward(self, x: torch.Tensor, return_mine: bool = False):
        if x.dtype == torch.uint8:  # u8 cell codes [N, H, W] (CNNResidualPolicy.forward)
            from .fused import codes_to_obs
            x = codes_to_obs(x)
        f = self.backbone(x)
        n = f.shape[0]
        logits = self.policy_head(f).reshape(n, -1)
        value = self.value_head(f).squeeze(-1)
        if return_mine:
            return logits, value, self.mine_head(f)  # not detached in the small model (cnn.py:55-57)
        return logits, value

    def beta_regularizer(self) -> torch.Tensor:
        return next(self.parameters()).new_zeros(())


def build_model(name: str, *, obs_shape: tuple[int, int, int], env_overrides: Dict[str, bool] | None = None,
                model_cfg: Optional[dict] = None) -> nn.Module:
    """models/__init__.py:17-49: 'cnn' | 'cnn_residual' | 'cnn_large'."""
    from . import exact_fp32_convs
    exact_fp32_convs()  # before the model's first (fp32, MIOpen) convolution
    cfg = dict(model_cfg or {})
    in_ch = obs_shape[0]
    if name == "cnn":
        return CNNPolicy(in_channels=in_ch, hidden=int(cfg.pop("hidden", 64)))
    if name in ("cnn_residual", "cnn_large"):
        return CNNResidualPolicy(in_ch, stem_channels=int(cfg.pop("stem_channels", 128)),
                                 blocks=int(cfg.pop("blocks", 6)), dropout=float(cfg.pop("dropout", 0.05)),
                                 value_hidden=int(cfg.pop("value_hidden", 256)))
    raise ValueError(f"Unknown model name: {name}")


def strip_compile_prefix(state_dict: dict) -> dict:
    """Checkpoints from torch.compile carry '_orig_mod.' (train_rl.py:405-406, eval.py:583-584)."""
    if any(k.startswith("_orig_mod.") for k in state_dict):
        return {k.replace("_orig_mod.", "", 1): v for k, v in state_dict.items()}
    return state_dict


__all__ = ["CNNPolicy", "CNNResidualPolicy", "build_model", "strip_compile_prefix"]

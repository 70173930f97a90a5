"""Policy/value/belief networks, state_dict-compatible with the reference.

Reference: minesweeper/models/cnn_residual.py:7-99 (CNNResidualPolicy),
minesweeper/models/cnn.py:7-60 (CNNPolicy), minesweeper/models/__init__.py:17-49
(build_model). Module attribute names, Sequential indices and parameter
creation order are the reference's, so (a) checkpoints load unchanged
(``stem.{0,1}``, ``residual_stack.{i}.{conv1,norm1,conv2,norm2}``,
``policy_head.{0,2}``, ``value_head.{2,4,6}``, ``mine_head.{0,2}``) and
(b) ``torch.manual_seed(s)`` yields bit-identical initial weights (checked
against tests/golden/model_full_*.npz).

MI355X notes: the 3x3 conv stack runs as MIOpen implicit-GEMM convolutions on
MFMA under bf16 autocast; ``channels_last()`` switches the
activations to NHWC, which MIOpen's MFMA conv kernels prefer.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


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

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.dropout(self.act(self.norm1(self.conv1(x))))
        y = self.norm2(self.conv2(y))
        return self.act(y + x)


class CNNResidualPolicy(nn.Module):
    """Residual CNN trunk + policy (per-cell logit), value (GAP MLP) and
    detached belief (per-cell mine logit) heads (cnn_residual.py:30-99)."""

    def __init__(self, in_channels: int, *, stem_channels: int = 128, blocks: int = 6,
                 dropout: float = 0.05, value_hidden: int = 256) -> None:
        super().__init__()
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

        # fused MFMA trunk (csrc/mscnn*.hip) on HIP devices under bf16 or fp16 autocast;
        # MS_AMD_FUSED=0 forces the PyTorch op chain (A/B measurements)
        self.fused = os.environ.get("MS_AMD_FUSED", "1") != "0"

    def set_gradient_checkpointing(self, enabled: bool) -> None:  # API parity (no-op, as the reference)
        return None

    def use_fused(self, x: torch.Tensor) -> bool:
        conv0 = self.stem[0]
        return (self.fused and x.is_cuda and conv0.out_channels == 96 and conv0.in_channels <= 16
                and x.shape[2] * x.shape[3] <= 512 and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") in (torch.bfloat16, torch.float16))

    def features(self, x: torch.Tensor) -> torch.Tensor:
        return self.residual_stack(self.stem(x))

    def _heads_nhwc(self, f: torch.Tensor, H: int, W: int, return_mine: bool):
        """The three heads on NHWC trunk features [N, H*W, C]: a 1x1 conv is a linear map
        over channels, so policy/mine heads are two GEMMs over N*H*W rows."""
        def pointwise(head, t):
            c0, c2 = head[0], head[2]
            h = F.relu(F.linear(t, c0.weight.flatten(1), c0.bias))
            return F.linear(h, c2.weight.flatten(1), c2.bias).squeeze(-1)
        n = f.shape[0]
        logits = pointwise(self.policy_head, f)  # [N, H*W], index r*W + c
        vh = self.value_head
        v = f.float().mean(1)  # AdaptiveAvgPool2d(1) + Flatten
        value = vh[6](F.relu(vh[4](F.relu(vh[2](v))))).squeeze(-1)
        if return_mine:
            return logits, value, pointwise(self.mine_head, f.detach()).view(n, 1, H, W)
        return logits, value

    def _heads_fused(self, f: torch.Tensor, H: int, W: int, return_mine: bool):
        """Heads through csrc/msheads.hip: policy + mine logits and the pooled features in
        one pass over f; the value MLP (N x 96 -> 1) stays a PyTorch op."""
        from .fused import heads_apply
        logits, pooled, mine = heads_apply(f, self.policy_head, self.mine_head if return_mine else None)
        vh = self.value_head
        value = vh[6](F.relu(vh[4](F.relu(vh[2](pooled))))).squeeze(-1)
        if return_mine:
            return logits, value, mine.view(f.shape[0], 1, H, W)
        return logits, value

    def forward(self, x: torch.Tensor, return_mine: bool = False):
        if self.use_fused(x):
            from .fused import fused_features
            f = fused_features(self, x, torch.get_autocast_dtype("cuda"))
            return self._heads_fused(f, x.shape[2], x.shape[3], return_mine)
        f = self.features(x)
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

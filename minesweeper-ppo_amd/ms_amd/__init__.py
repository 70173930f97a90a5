"""ms_amd — MI355X-native vectorised Minesweeper + PPO rollout engine.

Drop-in for the hot path of yakvrz/minesweeper-ppo: the batched
board step (HIP, libmsenv.so), on-device rollout storage + GAE, the residual
CNN policy under PyTorch-ROCm, and the PPO update with an RCCL gradient
all-reduce across ranks.
"""
import os as _os

# fp32 means fp32: MIOpen's Winograd solvers for fp32 3x3 convolutions give gradients of the
# shipped model ~130x further from a float64 computation than the reference's own fp32 CPU
# gradients (tools/grad_diag.py on MI355X); without them the error is <= 2x.
# The bf16 training path runs the fused kernels and never reaches MIOpen. Must be set before
# MIOpen's first convolution; an explicit user setting wins.
_os.environ.setdefault("MIOPEN_DEBUG_CONV_WINOGRAD", "0")

from .env import EnvConfig, VecMinesweeper, OBS_CHANNELS  # noqa: F401

__all__ = ["EnvConfig", "VecMinesweeper", "OBS_CHANNELS"]

"""ms_amd — MI355X-native vectorised Minesweeper + PPO rollout engine.

Drop-in for the hot path of yakvrz/minesweeper-ppo: the batched
board step (HIP, libmsenv.so), on-device rollout storage + GAE, the residual
CNN policy under PyTorch-ROCm, and the PPO update with an RCCL gradient
all-reduce across ranks.
"""
from .env import EnvConfig, VecMinesweeper, OBS_CHANNELS  # noqa: F401

__all__ = ["EnvConfig", "VecMinesweeper", "OBS_CHANNELS"]

"""ms_amd — MI355X-native vectorised Minesweeper + PPO rollout engine.

Drop-in for the hot path of yakvrz/minesweeper-ppo: the batched
board step (HIP, libmsenv.so), on-device rollout storage + GAE, the residual
CNN policy under PyTorch-ROCm, and the PPO update with an RCCL gradient
all-reduce across ranks.
"""
import logging as _logging
import os as _os

from .env import EnvConfig, VecMinesweeper, OBS_CHANNELS  # noqa: F401


def exact_fp32_convs() -> bool:
    """fp32 means fp32: MIOpen's Winograd solvers for fp32 3x3 convolutions give gradients of the
    shipped model ~130x further from a float64 computation than the reference's own fp32 CPU
    gradients (tools/grad_diag.py on MI355X); without them the error is <= 2x.
    Sets MIOPEN_DEBUG_CONV_WINOGRAD=0 unless the user chose a value, and logs it once. MIOpen
    reads it at its first convolution, so every model constructor of ms_amd.models calls this
    (a model built directly, as the reference's code builds it, got Winograd), as do
    ``build_model``, ``Trainer`` and ``evaluate_model``; importing ``ms_amd`` does not, so other
    models in the same process keep MIOpen's defaults unless one of those ran first (the setting
    is process-wide). The 16-bit training path runs the fused kernels and never
    reaches MIOpen. Returns True when the setting is in effect."""
    if "MIOPEN_DEBUG_CONV_WINOGRAD" not in _os.environ:
        _os.environ["MIOPEN_DEBUG_CONV_WINOGRAD"] = "0"
        _logging.getLogger("ms_amd").info("MIOPEN_DEBUG_CONV_WINOGRAD=0 (exact fp32 convolutions)")
    return _os.environ["MIOPEN_DEBUG_CONV_WINOGRAD"] == "0"


__all__ = ["EnvConfig", "VecMinesweeper", "OBS_CHANNELS", "exact_fp32_convs"]

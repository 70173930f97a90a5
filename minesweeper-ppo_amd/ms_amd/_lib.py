"""ctypes binding of libmsenv.so (the C ABI declared in include/msenv.h).

torch is imported first so that the HIP runtime torch ships is the one the
library binds to (both carry SONAME libamdhip64.so.7; the loader reuses the
already-mapped one). A second runtime in the process would make torch's
streams and pointers invalid for our kernels, so load() verifies that exactly
one libamdhip64 is mapped. There is no CPU fallback: if the library is
missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# MSENV_LIB may point at libmsenv_diag.so (tools/diag_step.py); default is the product build
LIB_PATH = os.environ.get("MSENV_LIB") or os.path.join(PKG_DIR, "libmsenv.so")
ABI_VERSION = 3

MS_OUTCOME_NONE, MS_OUTCOME_WIN, MS_OUTCOME_LOSS = 0, 1, 2
MS_TAPE_UNIFORM, MS_TAPE_SAFE_BIASED = 0, 1
MS_LATE_SHARED, MS_LATE_KEYED = 0, 1


class MsEnvError(RuntimeError):
    """Raised when a C ABI call returns a nonzero status."""


class MsCfg(ctypes.Structure):
    _fields_ = [("H", ctypes.c_int32), ("W", ctypes.c_int32), ("mine_count", ctypes.c_int32),
                ("guarantee_safe_neighborhood", ctypes.c_int32), ("win_reward", ctypes.c_double),
                ("loss_reward", ctypes.c_double), ("step_penalty", ctypes.c_double)]


_lib = None

# name -> argtypes (restype int unless listed in _RESTYPES)
_vp, _i64, _u64, _i32, _f32 = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int32,
                               ctypes.c_float)
SIGNATURES = {
    "ms_last_error": [],
    "ms_abi_version": [],
    "ms_create": [ctypes.POINTER(MsCfg), _i64, _u64, _i64, _i64, ctypes.POINTER(_vp)],
    "ms_destroy": [_vp],
    "ms_reset": [_vp, _vp, _vp, _vp],
    "ms_step": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "ms_step_i32": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "ms_step_codes": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "ms_labels": [_vp, _vp, _vp, _vp],
    "ms_snapshot": [_vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "ms_rng_state": [_vp, _vp, _vp],
    "ms_tape_actions": [_vp, _u64, _i32, _vp, _vp],
    "ms_run_tape": [_vp, _u64, _i32, _i32, _i32] + [_vp] * 10,
    "ms_gae": [_vp, _vp, _vp, _vp, _i32, _i64, _f32, _f32, _vp, _vp, _vp],
    "ms_sample_masked": [_vp, _vp, _i64, _i32, _i64, _u64, _u64, _vp, _vp, _vp],
    "ms_dropout_masks": [_vp, _i64, _i32, _i32, _u64, _u64, _f32, _vp, _vp],
    "ms_set_late_start": [_vp, ctypes.c_double, _i32, _i32, _i32, _i32, _u64],
    "ms_set_late_start_mode": [_vp, _i32],
    "ms_late_rng_state": [_vp, _vp],
    # msenv_debug.h
    "ms_set_debug_flags": [_vp, ctypes.c_uint32],
    "ms_set_diag": [_vp, _vp],
    "ms_set_timing_events": [_vp, _vp, _vp],
    "ms_event_create": [ctypes.POINTER(_vp)],
    "ms_event_elapsed_ms": [_vp, _vp, ctypes.POINTER(ctypes.c_float)],
    "ms_event_destroy": [_vp],
}
MS_DBG_FORCE_SERIAL_PLACEMENT = 1
MS_DBG_FORCE_CHAIN_PLACEMENT = 2
MS_DBG_ONE_BOARD_PER_WAVE = 4  # ms_step without the lane-packed small-board kernel
MS_DBG_TWO_BOARDS_PER_WAVE = 8  # the lane-packed kernel with 32-lane groups
MS_DBG_FORCE_PACKED = 16  # 16x16: the lane-packed kernel below its env-count threshold too
_RESTYPES = {"ms_last_error": ctypes.c_char_p, "ms_abi_version": ctypes.c_int32}


def _hip_runtimes_mapped() -> set[str]:
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    paths.add(os.path.realpath(line.split()[-1]))
    except OSError:
        pass
    return paths


def load():
    """Load libmsenv.so (once) and declare every C ABI signature."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MsEnvError(f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; g.build()'`"
                         " (or `make -C minesweeper-ppo_amd`)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    if lib.ms_abi_version() != ABI_VERSION:
        raise MsEnvError(f"libmsenv ABI {lib.ms_abi_version()} != expected {ABI_VERSION}")
    runtimes = _hip_runtimes_mapped()
    if len(runtimes) > 1:
        raise MsEnvError(f"more than one HIP runtime mapped in this process: {sorted(runtimes)}")
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != 0:
        raise MsEnvError(load().ms_last_error().decode(errors="replace"))


def ptr(t) -> int | None:
    """data_ptr of a tensor (None passes NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream

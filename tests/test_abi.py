"""CPU-side checks of the drop-in boundary: libmsenv.so loads, exports every
symbol include/msenv.h declares, and argument validation fails loudly."""
from __future__ import annotations

import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADERS = [os.path.join(ROOT, "include", h) for h in ("msenv.h", "msenv_debug.h")]
CNN_HEADER = os.path.join(ROOT, "include", "mscnn.h")


def header_functions(headers=HEADERS, prefix="ms_"):
    src = "".join(open(h).read() for h in headers)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(" + prefix + r"[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for name in ("ms_create", "ms_destroy", "ms_reset", "ms_step", "ms_step_i32", "ms_labels",
                 "ms_snapshot", "ms_tape_actions", "ms_gae", "ms_sample_masked", "ms_dropout_masks", "ms_last_error",
                 "ms_rng_state", "ms_abi_version"):
        assert name in fns


def test_library_exports_every_header_symbol():
    from ms_amd import _lib as L
    lib = L.load()
    for name in header_functions():
        assert hasattr(lib, name), name
        assert name in L.SIGNATURES, f"{name} has no ctypes signature"


def test_library_exports_every_cnn_header_symbol():
    from ms_amd import _lib as L
    lib = L.load()
    fns = header_functions([CNN_HEADER], "mc_")
    assert {"mc_conv_gn_fwd", "mc_conv_gn_bwd", "mc_conv_gn_bwd_workspace", "mc_heads_fwd", "mc_heads_bwd",
            "mc_heads_bwd_workspace", "mc_last_error"} <= set(fns)
    for name in fns:
        assert hasattr(lib, name), name


def test_library_exports_every_ppo_loss_header_symbol():
    from ms_amd import _lib as L
    lib = L.load()
    fns = header_functions([os.path.join(ROOT, "include", "msppo.h")], "mc_")
    assert {"mc_ppo_loss_workspace", "mc_ppo_loss_fwd", "mc_ppo_loss_bwd"} <= set(fns)
    for name in fns:
        assert hasattr(lib, name), name
    # ms_amd/loss.py's ctypes mirror of mc_ppo_loss_args has the C layout (12 pointers, 2 int32,
    # 8 floats, int64, int32 -> 152 bytes)
    from ms_amd.loss import _Args
    assert ctypes.sizeof(_Args) == 152 and _Args.M.offset == 136 and _Args.A.offset == 144
    ws = lib.mc_ppo_loss_workspace
    ws.restype, ws.argtypes = ctypes.c_int64, [ctypes.c_int64]
    assert ws(0) == -1 and ws(32768) == 2048 * 8 + 32768 * 4


def test_cnn_entry_points_validate_arguments():
    from ms_amd import _lib as L
    lib = L.load()
    lib.mc_last_error.restype = ctypes.c_char_p
    lib.mc_conv_gn_bwd_workspace.restype = ctypes.c_int64
    assert lib.mc_conv_gn_bwd_workspace(0, 16, 16, 96) == -1
    assert lib.mc_conv_gn_bwd_workspace(4, 16, 16, 32) == -1  # cin 16 or 96 only
    vp = ctypes.c_void_p
    i32 = ctypes.c_int32
    lib.mc_conv_gn_fwd.argtypes = [vp] * 11 + [i32] * 4 + [ctypes.c_float, i32, vp]
    assert lib.mc_conv_gn_fwd(*([None] * 11), 4, 16, 16, 96, 1e-5, 0, None) == 1
    assert b"bad argument" in lib.mc_last_error()
    # an unknown element type (include/mscnn.h: MC_DTYPE_BF16 0, MC_DTYPE_F16 1) is refused
    # before anything touches the device (the pointers are never dereferenced)
    fake = [vp(4096)] * 5 + [None, None, vp(4096), None, None, None]
    assert lib.mc_conv_gn_fwd(*fake, 4, 16, 16, 96, 1e-5, 2, None) == 1
    assert b"dtype 2" in lib.mc_last_error()
    lib.mc_heads_fwd.argtypes = [vp] * 7 + [ctypes.c_int64, i32, vp]
    assert lib.mc_heads_fwd(*([vp(4096)] * 6), None, 256, 7, None) == 1
    assert b"dtype 7" in lib.mc_last_error()


def test_trunk_entry_points_validate_arguments():
    """mc_trunk_fwd / mc_trunk_bwd / mc_conv_wgrad refuse bad layer lists and sizes before
    anything touches the device (the fake pointers are never dereferenced)."""
    from ms_amd import _lib as L
    from ms_amd import fused as F
    lib = L.load()
    lib.mc_last_error.restype = ctypes.c_char_p
    F._trunk_bind()
    fake = ctypes.c_void_p(4096)
    arr = (F._FwdLayer * 2)()
    assert F._tf(fake, arr, 1, None, 0, None, 4, 16, 16, 1e-5, 1, None) != 0  # odd layer count
    assert F._tf(fake, arr, 2, None, 0, None, 4, 16, 16, 1e-5, 1, None) != 0  # layer 0 has no weights
    assert b"layer 0" in lib.mc_last_error()
    for k in range(2):
        arr[k] = F._FwdLayer(4096, 4096, 4096, 4096, None, None, None, None, None)
    assert F._tf(fake, arr, 2, None, 0, None, 4, 16, 16, 1e-5, 1, None) != 0  # the last layer's out is required
    assert b"last layer" in lib.mc_last_error()
    arr[1] = F._FwdLayer(4096, 4096, 4096, 4096, 4096, 4096, None, None, None)
    assert F._tf(fake, arr, 2, None, 0, None, 4, 16, 16, 1e-5, 1, None) != 0  # dropout on a conv2
    assert F._tf(fake, arr, 17, None, 0, None, 4, 16, 16, 1e-5, 1, None) != 0  # > MC_TRUNK_MAX_LAYERS
    barr = (F._BwdLayer * 3)()
    assert F._tb(fake, barr, 2, fake, fake, 1 << 30, 4, 16, 16, 1, None) != 0  # even layer count
    assert F._tb(fake, barr, 3, fake, fake, 1 << 30, 4, 16, 16, 1, None) != 0  # empty layers
    assert b"layer 0" in lib.mc_last_error()
    barr[0] = F._BwdLayer(4096, 4096, 4096, 4096, None, 4096, 4096)  # the stem takes no wT
    assert F._tb(fake, barr, 3, fake, fake, 1 << 30, 4, 16, 16, 1, None) != 0
    assert F._tfws(4, 40, 40) < 0 and F._tbws(3, 4, 40, 40) < 0  # boards of more than 512 cells
    assert F._wg(fake, fake, fake, fake, 1 << 30, 4, 16, 16, 32, 1, None) != 0  # cin 16 or 96 only
    assert b"mc_conv_wgrad" in lib.mc_last_error()
    # mc_conv_wgrad_gn: y, stats, gamma, beta are required (dmask may be NULL)
    assert F._wgn(fake, None, fake, fake, fake, None, fake, fake, 1 << 30, 4, 16, 16, 1, None) != 0
    assert b"mc_conv_wgrad_gn: bad argument" in lib.mc_last_error()


def test_set_variant_validates_each_kernel_range():
    """mc_set_variant refuses a variant a kernel does not have (4 / 5 used to be
    accepted for every kernel and silently ran another kernel than the one named)."""
    from ms_amd import _lib as L
    lib = L.load()
    sv = lib.mc_set_variant
    sv.argtypes = [ctypes.c_int32, ctypes.c_int32]
    for kernel, vmax in ((0, 1), (1, 1), (2, 3), (3, 2)):
        for v in range(vmax + 1):
            assert sv(kernel, v) == 0
        assert sv(kernel, vmax + 1) != 0 and sv(kernel, -1) != 0
        assert sv(kernel, 0) == 0
    assert sv(4, 0) != 0


def test_single_hip_runtime_mapped():
    from ms_amd import _lib as L
    L.load()
    assert len(L._hip_runtimes_mapped()) == 1


def test_abi_version_and_error_paths():
    from ms_amd import _lib as L
    lib = L.load()
    assert lib.ms_abi_version() == L.ABI_VERSION
    h = ctypes.c_void_p()
    bad = L.MsCfg(100, 16, 40, 1, 1.0, -1.0, 1e-4)  # H > 64: rejected before any HIP call
    assert lib.ms_create(ctypes.byref(bad), 4, 0, 0, 4, ctypes.byref(h)) == 1
    assert b"unsupported board" in lib.ms_last_error()
    ok = L.MsCfg(16, 16, 40, 1, 1.0, -1.0, 1e-4)
    assert lib.ms_create(ctypes.byref(ok), 4, 0, 2, 4, ctypes.byref(h)) == 1  # range past n_total
    assert lib.ms_step(None, None, None, None, None, None, None, None, None, None, None) == 1
    assert b"null handle" in lib.ms_last_error()
    assert lib.ms_destroy(None) == 0
    with pytest.raises(L.MsEnvError):
        L.check(lib.ms_gae(None, None, None, None, 0, 0, 0.0, 0.0, None, None, None))


def test_envconfig_matches_reference_fields():
    from ms_amd import EnvConfig
    c = EnvConfig()
    assert (c.H, c.W, c.mine_count, c.guarantee_safe_neighborhood) == (8, 8, 10, True)
    assert (c.win_reward, c.loss_reward, c.step_penalty) == (1.0, -1.0, 1e-4)
    with pytest.raises(TypeError):
        EnvConfig(include_frontier_channel=True)  # unknown keys raise, as in env.py:19-30


def test_vec_refuses_cpu_device():
    from ms_amd import EnvConfig, VecMinesweeper
    from ms_amd._lib import MsEnvError
    with pytest.raises(MsEnvError):
        VecMinesweeper(4, EnvConfig(), device="cpu")

"""Timing experiments of the wave-specialised forward (libmsenv_wsx.so: `make libmsenv_wsx.so`,
-DMC_WSX, no phase stamps): the layer time at N = 32,768 with components removed (results are
garbage), to price each one.
    python tools/fwd_ws_exp.py [--variant 3] [--n 32768] [--lib diag|wsx]"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_lib_kind = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else "wsx"
os.environ["MSENV_LIB"] = os.path.join(ROOT, "minesweeper-ppo_amd", f"libmsenv_{_lib_kind}.so")
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=32768)
ap.add_argument("--variant", type=int, default=3)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--lib", default="wsx")
args = ap.parse_args()
import torch  # noqa: E402
from ms_amd import _lib as L  # noqa: E402
from ms_amd.fused import VARIANT_FWD, conv_gn_fwd, kernel_variant, prep_weight  # noqa: E402

n, H, W = args.n, 16, 16
dev = torch.device("cuda")
dt = torch.float16
x = (torch.randn(n, 256, 96, device=dev) * 0.5).to(dt)
wt = prep_weight(torch.randn(96, 96, 3, 3, device=dev) * 0.03, 96, dt)
b, g, be = torch.zeros(96, device=dev), torch.ones(96, device=dev), torch.zeros(96, device=dev)
res = torch.randn(n, 256, 96, device=dev).to(dt)
lib = L.load()
lib.mc_set_fwd_exp.argtypes = [ctypes.c_int32]
cases = [("full", 0), ("no MFMA", 1), ("no memory waves", 2), ("no weight streaming", 4), ("no stats", 8),
         ("no MFMA, no memory waves", 3), ("no weight streaming, no memory waves", 6),
         ("barriers + staging only (no MFMA, no mem, no weights, no stats)", 15)]


def t(fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / args.iters


with kernel_variant(VARIANT_FWD, args.variant):
    for rep in range(2):
        for name, e in cases:
            lib.mc_set_fwd_exp(e)
            ms = t(lambda: conv_gn_fwd(x, wt, b, g, be, H, W, res=res, want_mask=True)) * 1e3
            print(f"[variant {args.variant}] {name:62s} {ms:7.3f} ms", flush=True)
    lib.mc_set_fwd_exp(0)

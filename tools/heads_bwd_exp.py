"""Timing experiments of k_heads_bwd (libmsenv_wsx.so: `make libmsenv_wsx.so`, -DMC_WSX): the
launch time at M = 32,768 x 256 rows with parts removed (results are garbage), to price each.
    python tools/heads_bwd_exp.py [--n 32768] [--iters 20]"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MSENV_LIB"] = os.path.join(ROOT, "minesweeper-ppo_amd", "libmsenv_wsx.so")
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=32768)
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
import torch  # noqa: E402
from ms_amd import _lib as L  # noqa: E402
from ms_amd import fused  # noqa: E402

dev = torch.device("cuda")
n, P, C = args.n, 256, 96
M = n * P
dt = torch.float16
f = (torch.randn(n, P, C, device=dev) * 0.5).to(dt)
w1 = (torch.randn(192, C, device=dev) * 0.1).to(dt)
b1, w2 = torch.randn(192, device=dev) * 0.1, torch.randn(192, device=dev) * 0.1
dlp, dlm = torch.randn(n, P, device=dev), torch.randn(n, P, device=dev)
gadd = torch.randn(n, C, device=dev) / P
df = torch.empty_like(f)
dw1, db1, dw2 = torch.empty(192, C, device=dev), torch.empty(192, device=dev), torch.empty(192, device=dev)
lib = L.load()
fused._heads_bind()
nws = int(fused._hbws(M))
work = torch.empty(nws, device=dev)
lib.mc_set_heads_exp.argtypes = [ctypes.c_int32]
st = L.stream_ptr(dev)


def run():
    fused._check(fused._hb(L.ptr(f), L.ptr(dlp), L.ptr(dlm), L.ptr(w1), None, L.ptr(b1), L.ptr(w2), L.ptr(gadd), P,
                           L.ptr(df), L.ptr(dw1), L.ptr(db1), L.ptr(dw2), L.ptr(work), nws, M, 1, st))


cases = [("full", 0), ("no df stores", 1), ("no dW1 phase", 2), ("no H recompute MFMAs", 4), ("no f loads", 8),
         ("no dh LDS writes", 16), ("no df MFMAs", 32), ("no df MFMAs + stores", 33), ("only staging + H + dh (no df, dW1)", 35),
         ("only staging (no H, dh, df, dW1)", 63)]
for rep in range(2):
    for name, e in cases:
        lib.mc_set_heads_exp(e)
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            run()
        torch.cuda.synchronize()
        print(f"{name:40s} {(time.perf_counter() - t0) / args.iters * 1e3:7.3f} ms (incl. k_heads_reduce)", flush=True)
lib.mc_set_heads_exp(0)

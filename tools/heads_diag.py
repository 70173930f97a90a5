"""Diagnostic: phase cycle totals of k_heads_bwd (libmsenv_diag.so, MC_DIAG s_memtime stamps), per
wave and per 64-row tile, at one 16x16 PPO minibatch (M = 32,768 x 256 rows).
    python tools/heads_diag.py [--n 32768] [--P 256]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MSENV_LIB"] = os.path.join(ROOT, "minesweeper-ppo_amd", "libmsenv_diag.so")
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=32768)
ap.add_argument("--P", type=int, default=256)
args = ap.parse_args()
import torch  # noqa: E402
from ms_amd import _lib as L  # noqa: E402
from ms_amd import fused  # noqa: E402

dev = torch.device("cuda")
n, P, C = args.n, args.P, 96
M = n * P
f = (torch.randn(n, P, C, device=dev) * 0.5).to(torch.float16)
w1 = (torch.randn(192, C, device=dev) * 0.1).to(torch.float16)
b1, w2 = torch.randn(192, device=dev) * 0.1, torch.randn(192, device=dev) * 0.1
dlp, dlm = torch.randn(n, P, device=dev), torch.randn(n, P, device=dev)
gadd = torch.randn(n, C, device=dev) / P
df = torch.empty_like(f)
dw1, db1, dw2 = torch.empty(192, C, device=dev), torch.empty(192, device=dev), torch.empty(192, device=dev)
lib = L.load()
fused._heads_bind()
nws = int(fused._hbws(M))
work = torch.empty(nws, device=dev)
diag = torch.zeros(1024 * 4 * 8, dtype=torch.int64, device=dev)
lib.mc_set_heads_diag.argtypes = [ctypes.c_void_p]
st = L.stream_ptr(dev)


def run():
    fused._check(fused._hb(L.ptr(f), L.ptr(dlp), L.ptr(dlm), L.ptr(w1), None, L.ptr(b1), L.ptr(w2), L.ptr(gadd), P,
                           L.ptr(df), L.ptr(dw1), L.ptr(db1), L.ptr(dw2), L.ptr(work), nws, M, 1, st))


run()
torch.cuda.synchronize()
lib.mc_set_heads_diag(diag.data_ptr())
run()
torch.cuda.synchronize()
lib.mc_set_heads_diag(None)
d = diag.view(-1, 4, 8).cpu().double()
d = d[d.sum((1, 2)) > 0]
grid = d.shape[0]
tiles = (M + 63) // 64 / grid
names = {0: "DMA issue", 1: "vmcnt wait", 2: "3 barriers", 3: "H + dh", 4: "df + stage", 5: "dW1", 7: "df stores+loop"}
print(f"grid {grid}, {tiles:.1f} tiles per workgroup; s_memtime ticks per tile, waves 0..3:")
tot = [0.0] * 4
for k, nm in names.items():
    v = (d[:, :, k].mean(0) / tiles).tolist()
    tot = [a + b for a, b in zip(tot, v)]
    print(f"  {nm:16s} " + " ".join(f"{x:8.0f}" for x in v))
print(f"  {'total':16s} " + " ".join(f"{x:8.0f}" for x in tot))

"""Diagnostic: phase cycle totals of the fused forward kernel (libmsenv_diag.so, built
with -DMC_DIAG): stage input | 9 taps | GN stats | y->LDS | scale/shift+outputs | tail barrier.
Printed as s_memtime ticks per sample per workgroup (all workgroups run concurrently).
    python tools/fwd_diag.py [--n 32768] [--hw 16x16] [--pf 1]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MSENV_LIB"] = os.path.join(ROOT, "minesweeper-ppo_amd", "libmsenv_diag.so")
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=32768)
ap.add_argument("--hw", default="16x16")
ap.add_argument("--cin", type=int, default=96)
args = ap.parse_args()
import torch  # noqa: E402
from ms_amd import _lib as L  # noqa: E402
from ms_amd.fused import conv_gn_fwd, prep_weight  # noqa: E402

H, W = (int(v) for v in args.hw.split("x"))
n, P, cin = args.n, H * W, args.cin
dev = torch.device("cuda")
x = (torch.randn(n, P, cin, device=dev) * 0.5).to(torch.bfloat16)
w = torch.randn(96, cin, 3, 3, device=dev) * 0.03
b, g, be = torch.zeros(96, device=dev), torch.ones(96, device=dev), torch.zeros(96, device=dev)
res = torch.randn(n, P, 96, device=dev).to(torch.bfloat16) if cin == 96 else None
wt = prep_weight(w, cin)
diag = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
lib = L.load()
lib.mc_set_fwd_diag.argtypes = [ctypes.c_void_p]
conv_gn_fwd(x, wt, b, g, be, H, W, res=res)
torch.cuda.synchronize()
lib.mc_set_fwd_diag(diag.data_ptr())
conv_gn_fwd(x, wt, b, g, be, H, W, res=res)
torch.cuda.synchronize()
lib.mc_set_fwd_diag(None)
d = diag.view(-1, 8).cpu()
d = d[d.sum(1) > 0].double()
grid = d.shape[0]
per_sample = d.sum(0) / n * grid / grid  # ticks per sample (each WG processes n/grid samples)
per_wg_sample = d.mean(0) / (n / grid)
names = ["stage+w0", "9 taps", "GN stats", "y->LDS", "scale+out", "tail sync"]
print(f"grid {grid} workgroups, {n / grid:.1f} samples each; ticks per sample per workgroup:")
tot = 0.0
for i, nm in enumerate(names):
    print(f"  {nm:10s} {per_wg_sample[i]:9.0f}")
    tot += per_wg_sample[i]
print(f"  {'total':10s} {tot:9.0f}")

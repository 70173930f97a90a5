"""Diagnostic: where the wave-specialised forward (k_conv_gn_fwd_ws, libmsenv_diag.so built with
-DMC_DIAG) spends its time. Per segment (the stretch after each of the 11 barriers of an
iteration: taps 0..8, statistics pass 2, coefficients) the s_memtime ticks conv wave 0 and memory
wave 4 of every workgroup spent working and then waiting at the next barrier, per sample.
    python tools/fwd_ws_diag.py [--n 32768] [--hw 16x16] [--cin 96]"""
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
ap.add_argument("--dtype", default="fp16")
ap.add_argument("--variant", type=int, default=2, help="2: s_barrier form, 3: grp_bar form")
args = ap.parse_args()
import torch  # noqa: E402
from ms_amd import _lib as L  # noqa: E402
from ms_amd.fused import VARIANT_FWD, conv_gn_fwd, kernel_variant, prep_weight  # noqa: E402

H, W = (int(v) for v in args.hw.split("x"))
n, P, cin = args.n, H * W, args.cin
dt = torch.float16 if args.dtype == "fp16" else torch.bfloat16
dev = torch.device("cuda")
x = (torch.randn(n, P, cin, device=dev) * 0.5).to(dt)
w = torch.randn(96, cin, 3, 3, device=dev) * 0.03
b, g, be = torch.zeros(96, device=dev), torch.ones(96, device=dev), torch.zeros(96, device=dev)
res = torch.randn(n, P, 96, device=dev).to(dt) if cin == 96 else None
wt = prep_weight(w, cin, dt)
diag = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
lib = L.load()
lib.mc_set_fwd_diag.argtypes = [ctypes.c_void_p]
with kernel_variant(VARIANT_FWD, args.variant):
    for _ in range(2):
        conv_gn_fwd(x, wt, b, g, be, H, W, res=res, want_mask=True)
    torch.cuda.synchronize()
    lib.mc_set_fwd_diag(diag.data_ptr())
    conv_gn_fwd(x, wt, b, g, be, H, W, res=res, want_mask=True)
    torch.cuda.synchronize()
    lib.mc_set_fwd_diag(None)
d = diag[: (diag.numel() // 48) * 48].view(-1, 2, 24).cpu().double()
d = d[d[:, 0].sum(1) > 0]
grid = d.shape[0]
per = d.mean(0) / (n / grid)  # ticks per sample per workgroup
segs = [f"tap {k}" for k in range(9)] + ["stats p2", "coef/next"]
if args.variant == 3:  # grp_bar form: the memory waves' segment 0 = epilogue, segment 10 = staging + loads
    segs[0] = "tap 0 | mem: epilogue"
    segs[10] = "coef | mem: x, loads"
print(f"grid {grid} workgroups, {n / grid:.1f} samples each; s_memtime ticks per sample:")
print(f"{'segment':10s} {'conv work':>10s} {'conv wait':>10s} {'mem work':>10s} {'mem wait':>10s}")
tot = torch.zeros(4, dtype=torch.float64)
for k in range(11):
    row = torch.tensor([per[0, k], per[0, 12 + k], per[1, k], per[1, 12 + k]])
    tot += row
    print(f"{segs[k]:10s} " + " ".join(f"{v:10.0f}" for v in row))
print(f"{'total':10s} " + " ".join(f"{v:10.0f}" for v in tot))

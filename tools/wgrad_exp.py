"""Timing experiments of k_wgrad (libmsenv_wsx.so: `make libmsenv_wsx.so`, -DMC_WSX): each WGX_*
bit removes one part of the kernel (results wrong), so its cost reads off the launch time under
`rocprofv3 --kernel-trace --stats`. N = 32,768 samples of 16x16 boards, 96 -> 96 channels, bf16.
Bits: 1 = no LDS staging (no prefetch loads, no LDS writes), 2 = no MFMA loop, 4 = no barriers,
8 = every prefetch loads the workgroup's first sample again (L2-resident; k_wgrad only).
Argument 2: the k_wgrad variant (2 = k_wgrad with the pinned schedule, 3 = k_wgrad_c96).
The launches of one setting are labelled in the log in run order (8 per setting)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
os.environ["MSENV_LIB"] = os.path.join(ROOT, "minesweeper-ppo_amd", "libmsenv_wsx.so")
import torch  # noqa: E402

from ms_amd import _lib  # noqa: E402
from ms_amd.fused import VARIANT_WGRAD, conv_gn_bwd, conv_gn_fwd, kernel_variant, prep_weight, prep_weight_t  # noqa: E402

lib = _lib.load()
lib.mc_set_wgrad_exp.argtypes = [ctypes.c_int32]
dev = torch.device("cuda")
n, H, W, cin, P = 32768, 16, 16, 96, 256
dt = torch.bfloat16
torch.manual_seed(0)
x = (torch.randn(n, P, cin, device=dev) * 0.5).to(dt)
w = torch.randn(96, cin, 3, 3, device=dev) * 0.03
b, g, be = torch.zeros(96, device=dev), torch.ones(96, device=dev), torch.zeros(96, device=dev)
out, y, st, rm = conv_gn_fwd(x, prep_weight(w, cin, dt), b, g, be, H, W, want_mask=True)
dout = torch.randn(n, P, 96, device=dev).to(dt)
wT = prep_weight_t(w, dt)
exps = [int(e) for e in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4,5").split(",")]
var = int(sys.argv[2]) if len(sys.argv) > 2 else 2
for e in exps:
    lib.mc_set_wgrad_exp(e)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    with kernel_variant(VARIANT_WGRAD, var):
        for _ in range(8):
            conv_gn_bwd(dout, None, y, st, g, x, H, W, wT=wT, rmask=rm)
    torch.cuda.synchronize()
    print(f"exp {e}: 8 launches issued", flush=True)
lib.mc_set_wgrad_exp(0)

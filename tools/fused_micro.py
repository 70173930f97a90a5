"""Time the fused conv+GN+ReLU MFMA kernel against the PyTorch (MIOpen) chain
for one layer at the PPO minibatch size. python tools/fused_micro.py [--n 32768]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from ms_amd.fused import (VARIANT_BWD, VARIANT_FWD, conv_gn_bwd, conv_gn_fwd, kernel_variant,  # noqa: E402
                          prep_weight, prep_weight_t)

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=32768)
ap.add_argument("--hw", default="16x16")
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--no-torch", action="store_true")
ap.add_argument("--bwd", action="store_true", help="also time the fused backward of the layer")
ap.add_argument("--mask", action="store_true", help="the forward also writes the ReLU bitmask (as training does)")
ap.add_argument("--variants", default="0", help="comma list of mc_set_variant values to time in turn "
                "(0 dispatcher, 1 per-sample, 2 wave-specialised), e.g. 1,2,1,2")
args = ap.parse_args()
H, W = (int(v) for v in args.hw.split("x"))
dev = torch.device("cuda")
n, P = args.n, H * W
x = (torch.randn(n, P, 96, device=dev) * 0.5).to(torch.bfloat16)
w = torch.randn(96, 96, 3, 3, device=dev) * 0.03
b, g, be = torch.zeros(96, device=dev), torch.ones(96, device=dev), torch.zeros(96, device=dev)
wt = prep_weight(w, 96)
res = torch.randn(n, P, 96, device=dev).to(torch.bfloat16)


def t(fn, iters):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


flop = 2 * n * P * 96 * 864
for var in (int(v) for v in args.variants.split(",")):
    with kernel_variant(VARIANT_FWD, var), kernel_variant(VARIANT_BWD, var):
        f1 = t(lambda: conv_gn_fwd(x, wt, b, g, be, H, W, res=res, want_mask=args.mask), args.iters)
        print(f"[variant {var}] fused conv+GN+res+ReLU  n={n} {H}x{W}: {f1 * 1e3:.3f} ms  "
              f"{flop / f1 / 1e12:.0f} TFLOP/s(conv)", flush=True)
        if args.bwd:  # the trainer's path: the forward's ReLU bitmask, the skip addend, dz kept
            out, y, st, rm = conv_gn_fwd(x, wt, b, g, be, H, W, res=res, want_mask=True)
            dout = torch.randn_like(out)
            wT = prep_weight_t(w)
            fb = t(lambda: conv_gn_bwd(dout, None, y, st, g, x, H, W, wT=wT, addend=res, want_dz=True, rmask=rm),
                   args.iters)
            print(f"[variant {var}] fused bwd (GN-bwd + dgrad + wgrad) n={n} {H}x{W}: {fb * 1e3:.3f} ms  "
                  f"{2 * flop / fb / 1e12:.0f} TFLOP/s", flush=True)
if args.no_torch:
    sys.exit(0)
xn = x.float().view(n, H, W, 96).permute(0, 3, 1, 2).contiguous().to(torch.bfloat16)
rn = res.float().view(n, H, W, 96).permute(0, 3, 1, 2).contiguous().to(torch.bfloat16)
conv = torch.nn.Conv2d(96, 96, 3, padding=1).to(dev)
gn = torch.nn.GroupNorm(6, 96).to(dev)


def torch_chain():
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        return torch.relu(gn(conv(xn)) + rn)


f2 = t(torch_chain, args.iters)
print(f"torch conv+GN+res+ReLU (bf16 autocast, NCHW): {f2 * 1e3:.2f} ms  {flop / f2 / 1e12:.0f} TFLOP/s  "
      f"speedup {f2 / f1:.2f}x", flush=True)

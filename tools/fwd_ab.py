"""Same-process A/B of the two forward kernels of one 96->96 layer (16x16 boards):
mc_set_fwd_impl auto (weight-resident, wave-specialised) vs per_sample, per mode
(residual / dropout / plain) and element type, with the two outputs compared.
python tools/fwd_ab.py [--n 32768] [--iters 20]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
import torch  # noqa: E402
from ms_amd.fused import conv_gn_fwd, prep_weight, set_fwd_impl  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=32768)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--dtypes", default="fp16,bf16")
ap.add_argument("--modes", default="res,dropout,plain")
args = ap.parse_args()
dev = torch.device("cuda")
n, H, W, P = args.n, 16, 16, 256
torch.manual_seed(0)
flop = 2 * n * P * 96 * 864


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for dt in [{"fp16": torch.float16, "bf16": torch.bfloat16}[d] for d in args.dtypes.split(",")]:
    x = (torch.randn(n, P, 96, device=dev) * 0.5).to(dt)
    w = torch.randn(96, 96, 3, 3, device=dev) * 0.03
    b, g, be = torch.randn(96, device=dev) * 0.1, 1 + 0.1 * torch.randn(96, device=dev), 0.1 * torch.randn(96, device=dev)
    wt = prep_weight(w, 96, dt)
    res = torch.randn(n, P, 96, device=dev).to(dt)
    dm = (torch.rand(n, 96, device=dev) > 0.05).float() / 0.95
    for mode, kw in [(m, {"res": dict(res=res), "dropout": dict(dmask=dm), "plain": {}}[m])
                     for m in args.modes.split(",")]:
        outs, times = {}, {"auto": [], "per_sample": []}
        for rep in range(args.reps):
            for impl in ("per_sample", "auto"):
                set_fwd_impl(impl)
                f = lambda: conv_gn_fwd(x, wt, b, g, be, H, W, want_mask=True, **kw)  # noqa: E731
                times[impl].append(timed(f, args.iters))
                if rep == 0:
                    outs[impl] = f()
        set_fwd_impl("auto")
        o_a, y_a, s_a, m_a = outs["auto"]
        o_p, y_p, s_p, m_p = outs["per_sample"]
        dy = (y_a.float() - y_p.float()).abs().max().item()
        do = ((o_a.float() - o_p.float()).norm() / o_p.float().norm()).item()
        ds = (s_a - s_p).abs().max().item()
        dmk = (m_a != m_p).float().mean().item()
        ta, tp = min(times["auto"]), min(times["per_sample"])
        print(f"{str(dt)[6:]:8s} {mode:8s} per_sample {tp:.3f} ms  auto {ta:.3f} ms  ({tp / ta:.2f}x, "
              f"{flop / ta / 1e9:.0f} TFLOP/s)  |dy|max {dy:.2e} out relL2 {do:.2e} |dstats| {ds:.2e} "
              f"mask diff {dmk:.2e}", flush=True)

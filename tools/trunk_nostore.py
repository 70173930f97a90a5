"""Timing experiment (libmsenv_diag.so only): is the one-launch trunk held up by its own global
stores? mc_set_trunk_dflags(1) drops the forward epilogue's stores (y, out, ReLU bits) and the
backward pass 2's stores (dy, skip slot); outputs are then garbage, the timing is what counts.
Alternates flags 0 / 1 in one process, HIP events around the training forward and the backward.
    python tools/trunk_nostore.py [--n 32768] [--hw 16x16] [--iters 10] [--rounds 3]"""
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
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--flags", default="0,1")
args = ap.parse_args()
import torch  # noqa: E402
from ms_amd import _lib as L  # noqa: E402
from ms_amd import fused as F  # noqa: E402
from ms_amd.models import CNNResidualPolicy  # noqa: E402

H, W = map(int, args.hw.split("x"))
dev = torch.device("cuda")
dt = torch.float16
torch.manual_seed(0)
m = CNNResidualPolicy(10, stem_channels=96, blocks=5, dropout=0.05, value_hidden=256).to(dev).train()
idx = torch.randint(0, 10, (args.n, H, W), device=dev)
obs = torch.nn.functional.one_hot(idx, 10).permute(0, 3, 1, 2).float().contiguous()
dms = [((torch.rand(args.n, 96, device=dev) >= 0.05).float() / 0.95).contiguous() for _ in range(5)]
df = torch.randn(args.n, H * W, 96, device=dev).to(dt)
lib = L.load()
lib.mc_set_trunk_dflags.argtypes = [ctypes.c_int]


def run(flags):
    lib.mc_set_trunk_dflags(flags)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = tn = 0.0
    for it in range(args.iters + 2):
        m.zero_grad(set_to_none=True)
        ev[0].record()
        f = F.fused_features(m, obs, dt, dmasks=dms)
        ev[1].record()
        f.backward(df)
        ev[2].record()
        torch.cuda.synchronize()
        if it >= 2:
            tf += ev[0].elapsed_time(ev[1])
            tb += ev[1].elapsed_time(ev[2])
        with torch.no_grad():
            ev[0].record()
            F.fused_features(m, obs, dt, dmasks=dms)
            ev[1].record()
        torch.cuda.synchronize()
        if it >= 2:
            tn += ev[0].elapsed_time(ev[1])
    lib.mc_set_trunk_dflags(0)
    k = args.iters
    return tf / k, tb / k, tn / k


fl = [int(x) for x in args.flags.split(",")]
for r in range(args.rounds):
    for f in fl:
        a, b, c = run(f)
        print(f"round {r} flags {f}: training fwd {a:.2f} ms, bwd (trunk + wgrad + stem) {b:.2f} ms, "
              f"no-grad fwd {c:.2f} ms", flush=True)

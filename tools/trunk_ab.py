"""Same-process A/B of the trunk (stem + residual stack) forward + backward: the one-launch
kernels (mc_trunk_fwd / mc_trunk_bwd + mc_conv_wgrad) against the per-layer kernels, and the
no-grad forward (the rollout's), at one PPO minibatch of the shipped model.
    python tools/trunk_ab.py [--n 32768] [--hw 16x16] [--iters 10] [--dtype fp16]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=32768)
ap.add_argument("--hw", default="16x16")
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--dtype", default="fp16")
ap.add_argument("--blocks", type=int, default=5)
ap.add_argument("--rounds", type=int, default=3)
args = ap.parse_args()
from ms_amd import fused as F  # noqa: E402
from ms_amd.models import CNNResidualPolicy  # noqa: E402

H, W = map(int, args.hw.split("x"))
dev = torch.device("cuda")
dt = {"fp16": torch.float16, "bf16": torch.bfloat16}[args.dtype]
torch.manual_seed(0)
m = CNNResidualPolicy(10, stem_channels=96, blocks=args.blocks, dropout=0.05, value_hidden=256).to(dev).train()
idx = torch.randint(0, 10, (args.n, H, W), device=dev)
obs = torch.nn.functional.one_hot(idx, 10).permute(0, 3, 1, 2).float().contiguous()
dms = [((torch.rand(args.n, 96, device=dev) >= 0.05).float() / 0.95).contiguous() for _ in range(args.blocks)]
df = torch.randn(args.n, H * W, 96, device=dev).to(dt)


def fwd_bwd():
    m.zero_grad(set_to_none=True)
    f = F.fused_features(m, obs, dt, dmasks=dms)
    f.backward(df)


def fwd_nograd():
    with torch.no_grad():
        F.fused_features(m, obs, dt, dmasks=dms)


def timeit(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / args.iters


for r in range(args.rounds):
    for chain in (True, False):
        with F.chain_path(chain):
            t1 = timeit(fwd_bwd)
            t0 = timeit(fwd_nograd)
        print(f"round {r} chain={int(chain)} n={args.n} {H}x{W} {args.dtype}: fwd+bwd {t1:.2f} ms, "
              f"no-grad fwd {t0:.2f} ms", flush=True)

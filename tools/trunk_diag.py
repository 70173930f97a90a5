"""Diagnostic: phase cycle totals of the one-launch trunk kernels (libmsenv_diag.so, MC_DIAG
s_memtime stamps) at one PPO minibatch of the shipped 96x5 model, in ticks per sample and layer
(average over workgroups, per wave).
    python tools/trunk_diag.py [--n 32768] [--hw 16x16]"""
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
lib.mc_set_trunk_diag.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
dfw = torch.zeros(1024 * 4 * 8, dtype=torch.int64, device=dev)
dbw = torch.zeros(1024 * 4 * 8, dtype=torch.int64, device=dev)


def step():
    m.zero_grad(set_to_none=True)
    f = F.fused_features(m, obs, dt, dmasks=dms)
    f.backward(df)


step()
torch.cuda.synchronize()
lib.mc_set_trunk_diag(dfw.data_ptr(), dbw.data_ptr())
step()
torch.cuda.synchronize()
lib.mc_set_trunk_diag(None, None)
for name, d, nl, phases in (("k_trunk_fwd", dfw, 10, ["top/stage", "9 taps", "GN stats", "y->LDS+coef", "epilogue"]),
                            ("k_trunk_bwd", dbw, 11, ["pass 1", "sums+coef", "pass 2", "dgrad taps", "dx->LDS"])):
    t = d.view(-1, 4, 8).cpu().double()
    t = t[t.sum((1, 2)) > 0]
    grid = t.shape[0]
    per = args.n / grid * nl
    print(f"{name}: grid {grid}, {args.n / grid:.1f} samples x {nl} layers per workgroup; ticks per sample-layer, waves 0..3")
    tot = [0.0] * 4
    for k, nm in enumerate(phases):
        v = (t[:, :, k].mean(0) / per).tolist()
        tot = [a + b for a, b in zip(tot, v)]
        print(f"  {nm:14s} " + " ".join(f"{x:8.0f}" for x in v))
    print(f"  {'total':14s} " + " ".join(f"{x:8.0f}" for x in tot))

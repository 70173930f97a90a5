"""Diagnostic: where k_trunk_fwd_pp's half-periods go (libmsenv_diag.so, MC_DIAG s_memtime stamps),
per wave of the 512-thread workgroup (waves 0-3 team A, 4-7 team B), averaged over workgroups:
MFMA-phase issue + taps and its waits + barriers per active tap interval; P0-P2 work and barrier
waits and the epilogue pieces' work and waits per active piece interval.
    python tools/trunk_pp_diag.py [--n 32768] [--hw 16x16] [--nograd]"""
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
ap.add_argument("--nograd", action="store_true")
ap.add_argument("--dflags", type=int, default=0, help="1: drop the epilogue stores, 2: drop the residual loads")
ap.add_argument("--variant", type=int, default=0, help="MCV_TRUNK_FWD variant: 0 lockstep, 2 ping-pong")
args = ap.parse_args()
import torch  # noqa: E402
from ms_amd import _lib as L  # noqa: E402
from ms_amd import fused as F  # noqa: E402
from ms_amd.models import CNNResidualPolicy  # noqa: E402

H, W = map(int, args.hw.split("x"))
dev = torch.device("cuda")
torch.manual_seed(0)
m = CNNResidualPolicy(10, stem_channels=96, blocks=5, dropout=0.05, value_hidden=256).to(dev).train()
idx = torch.randint(0, 10, (args.n, H, W), device=dev)
obs = torch.nn.functional.one_hot(idx, 10).permute(0, 3, 1, 2).float().contiguous()
dms = [((torch.rand(args.n, 96, device=dev) >= 0.05).float() / 0.95).contiguous() for _ in range(5)]
lib = L.load()
lib.mc_set_trunk_diag.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
dfw = torch.zeros(1024 * 8 * 8, dtype=torch.int64, device=dev)


def fwd():
    with torch.set_grad_enabled(not args.nograd):
        f = F.fused_features(m, obs, torch.float16, dmasks=dms)
    return f


fwd()
torch.cuda.synchronize()
lib.mc_set_trunk_dflags.argtypes = [ctypes.c_int]
lib.mc_set_trunk_dflags(args.dflags)
F.kernel_variant(F.VARIANT_TRUNK_FWD, args.variant).__enter__()
lib.mc_set_trunk_diag(dfw.data_ptr(), None)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
f = fwd()
e1.record()
torch.cuda.synchronize()
lib.mc_set_trunk_diag(None, None)
lib.mc_set_trunk_dflags(0)
print(f"variant {args.variant} dflags {args.dflags}: forward {'no-grad' if args.nograd else 'training'} {e0.elapsed_time(e1):.2f} ms (diag build)")
t = dfw.view(1024, 8, 8).cpu().double()
t = t[t.sum((1, 2)) > 0]
print(f"workgroups {t.shape[0]}")
a = t.mean(0)  # [8 waves][8]
names = ["mfma issue+taps", "mfma wait+bar", "P0-P2 work", "P0-P2 bar", "pieces work", "pieces bar"]
print("per active interval (ticks); columns waves 0..7")
for k, nm in enumerate(names):
    den = a[:, 6] if k < 2 else (a[:, 6] / 9 * 3 if k < 4 else a[:, 7])
    print(f"  {nm:16s} " + " ".join(f"{(a[w, k] / max(den[w].item(), 1)):8.0f}" for w in range(8)))
print("  totals (Mticks)  " + " ".join(f"{a[w, :6].sum().item() / 1e6:8.2f}" for w in range(8)))
print("  active tap intervals / pieces: " + " ".join(f"{a[w, 6].item():.0f}/{a[w, 7].item():.0f}" for w in range(8)))

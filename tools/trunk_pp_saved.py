"""Debug: the saved tensors of the one-launch trunk forward (y, stats, ReLU bits, outputs) under
k_trunk_fwd_pp (variants 0 / 2) against k_trunk_fwd2 (variant 1).
    python tools/trunk_pp_saved.py [--n 300] [--hw 16x16]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=300)
ap.add_argument("--hw", default="16x16")
args = ap.parse_args()
import torch  # noqa: E402
from ms_amd import fused as F  # noqa: E402
from ms_amd.models import CNNResidualPolicy  # noqa: E402

H, W = map(int, args.hw.split("x"))
dev = torch.device("cuda")
torch.manual_seed(0)
m = CNNResidualPolicy(10, stem_channels=96, blocks=2, dropout=0.05, value_hidden=64).to(dev).train()
idx = torch.randint(0, 10, (args.n, H, W), device=dev)
obs = torch.nn.functional.one_hot(idx, 10).permute(0, 3, 1, 2).float().contiguous()
dms = [((torch.rand(args.n, 96, device=dev) >= 0.05).float() / 0.95).contiguous() for _ in range(2)]
layers = F.trunk_layers(m)
x0 = F.obs_to_nhwc(obs, 16, torch.float16)
res = {}
for v in (1, 0, 2):
    with F.kernel_variant(F.VARIANT_TRUNK_FWD, v):
        res[v] = F._trunk_forward(x0, layers, H, W, dms, save=True)
    torch.cuda.synchronize()
ref = res[1]
for v in (0, 2):
    out, acts, ys, sts, rms = res[v]
    print(f"variant {v}: out max|d| {(out.float() - ref[0].float()).abs().max().item():.3e}")
    for li in range(len(ys)):
        d_y = (ys[li].float() - ref[2][li].float()).abs().max().item()
        d_s = (sts[li] - ref[3][li]).abs().max().item()
        nb = (rms[li] != ref[4][li]).sum().item()
        bits = torch.bitwise_xor(rms[li], ref[4][li])
        print(f"  layer {li}: y max|d| {d_y:.3e}, stats max|d| {d_s:.3e}, relu bytes differing {nb} "
              f"of {rms[li].numel()}; first bad {bits.nonzero()[:3].tolist() if nb else []}, "
              f"pp {rms[li].flatten()[:12].tolist()} ref {ref[4][li].flatten()[:12].tolist()}")

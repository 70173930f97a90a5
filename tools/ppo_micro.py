"""Micro-benchmark of one PPO minibatch update (fwd+bwd+AdamW) of the shipped
model on synthetic 16x16 observations: where does the combined loop's time go?
    python tools/ppo_micro.py --mb 32768 [--channels-last] [--benchmark] [--amp fp16|bf16|fp32]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mb", type=int, default=32768)
ap.add_argument("--iters", type=int, default=6)
ap.add_argument("--channels-last", action="store_true")
ap.add_argument("--benchmark", action="store_true")
ap.add_argument("--amp", default="fp16")
ap.add_argument("--fwd-only", action="store_true")
ap.add_argument("--chain", type=int, default=1, help="one-launch trunk (1) or per-layer kernels (0)")
ap.add_argument("--pure-bf16", action="store_true", help="model + obs in bf16, no autocast (timing only)")
ap.add_argument("--no-wgrad-gn", action="store_true", help="write conv1 outputs instead of recomputing them")
ap.add_argument("--value-splitk", type=int, default=32, help="fused.VALUE_SPLITK (0: autocast's Linear chain)")
ap.add_argument("--torch-prof", type=int, default=0, help="print the device time of N minibatches by aten op")
ap.add_argument("--foreach-adamw", action="store_true", help="torch's foreach AdamW instead of the fused kernel")
args = ap.parse_args()
torch.backends.cudnn.benchmark = args.benchmark
from ms_amd import fused as _F  # noqa: E402
from ms_amd.models import build_model  # noqa: E402
_F.CHAIN = bool(args.chain)
_F.WGRAD_GN = not args.no_wgrad_gn
_F.VALUE_SPLITK = args.value_splitk
from ms_amd.ppo import PPOConfig, ppo_update  # noqa: E402
from ms_amd.buffers import Batch  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
m = build_model("cnn_residual", obs_shape=(10, 16, 16),
                model_cfg=dict(stem_channels=96, blocks=5, dropout=0.05, value_hidden=256)).to(dev)
if args.pure_bf16:
    m = m.to(torch.bfloat16)
if args.channels_last:
    m = m.to(memory_format=torch.channels_last)
opt = torch.optim.AdamW(m.parameters(), lr=3e-4, fused=not args.foreach_adamw)  # as the Trainer
M = args.mb
g = torch.Generator(device=dev).manual_seed(0)
rev = torch.rand(M, 16, 16, device=dev, generator=g) < 0.4
cnt = torch.randint(0, 9, (M, 16, 16), device=dev, generator=g)
obs = torch.zeros(M, 10, 16, 16, device=dev)
obs[:, 0] = rev.float()
obs.scatter_(1, (1 + cnt).unsqueeze(1), rev.float().unsqueeze(1))
if args.pure_bf16:
    obs = obs.to(torch.bfloat16)
if args.channels_last:
    obs = obs.contiguous(memory_format=torch.channels_last)
mask = ~rev.view(M, -1)
acts = torch.multinomial(mask.float() + 1e-6, 1, generator=g).squeeze(1)
b = Batch(obs=obs, action_mask=mask, actions=acts, old_logp=-torch.rand(M, device=dev) * 5,
          values=torch.randn(M, device=dev), advantages=torch.randn(M, device=dev),
          returns=torch.randn(M, device=dev), mine_labels=(torch.rand(M, 16, 16, device=dev) < 0.15).float(),
          mine_valid=~rev)
cfg = PPOConfig(aux_mine_weight=0.05, aux_mine_calib_weight=0.01)
amp = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": None}[args.amp]
if args.pure_bf16:
    amp = None
    b.mine_labels = b.mine_labels.bfloat16()
scaler = torch.amp.GradScaler("cuda") if amp == torch.float16 else None  # the reference's fp16 path


def step():
    if args.fwd_only:
        with torch.no_grad(), torch.autocast("cuda", dtype=amp, enabled=amp is not None):
            m(obs)
    else:
        ppo_update(m, opt, b, cfg, scaler, amp_dtype=amp, sync_stats=False)


for _ in range(2):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(args.iters):
    step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / args.iters
gf = (0.4388 if args.fwd_only else 1.3073) * M
print(f"mb={M} cl={args.channels_last} bench={args.benchmark} amp={args.amp} fwd_only={args.fwd_only}: "
      f"{dt * 1e3:.1f} ms/iter, {gf / dt / 1e3:.1f} TFLOP/s, mem {torch.cuda.max_memory_allocated() / 1e9:.1f} GB")

if args.torch_prof:
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(args.torch_prof):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_device_time_total", row_limit=60,
                                                             max_name_column_width=40, max_shapes_column_width=70))

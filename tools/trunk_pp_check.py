"""Ping-pong trunk forward (k_trunk_fwd_pp, MCV_TRUNK_FWD variant 2) against the lockstep kernel
(k_trunk_fwd2, variant 1, bitwise the per-layer path): features, every parameter gradient (the
backward runs on each forward's saved y / stats / ReLU bits) and the pooled mean, as relative L2
errors and max |diff|; then same-process timing of the default (0: k_trunk_fwd_pp without saves,
k_trunk_fwd2 with) and both forced variants at one PPO minibatch.
    python tools/trunk_pp_check.py [--time-n 32768] [--iters 10]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("--time-n", type=int, default=32768)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--skip-check", action="store_true")
args = ap.parse_args()
import torch  # noqa: E402
from ms_amd import fused as F  # noqa: E402
from ms_amd.models import CNNResidualPolicy  # noqa: E402

dev = torch.device("cuda")


def model(blocks, seed=0):
    torch.manual_seed(seed)
    m = CNNResidualPolicy(10, stem_channels=96, blocks=blocks, dropout=0.05, value_hidden=64).to(dev).train()
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.GroupNorm):
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.3, 0.3)
    return m


def obs_(n, H, W, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    idx = torch.randint(0, 10, (n, H, W), device=dev, generator=g)
    return torch.nn.functional.one_hot(idx, 10).permute(0, 3, 1, 2).float().contiguous()


def dmasks(blocks, n, p=0.05):
    g = torch.Generator(device=dev).manual_seed(7)
    return [((torch.rand(n, 96, device=dev, generator=g) >= p).float() / (1.0 - p)).contiguous() for _ in range(blocks)]


def run(m, obs, dt, dms, variant, grad=True, chain=True):
    with F.kernel_variant(F.VARIANT_TRUNK_FWD, variant), F.chain_path(chain):
        m.zero_grad(set_to_none=True)
        if not grad:
            with torch.no_grad():
                f, pooled = F.fused_features(m, obs, dt, dmasks=dms, with_pooled=True)
            return f, pooled, None
        f, pooled = F.fused_features(m, obs, dt, dmasks=dms, with_pooled=True)
        g = torch.Generator(device=dev).manual_seed(3)
        df = torch.randn(f.shape, device=dev, generator=g).to(dt)
        f.backward(df)
        torch.cuda.synchronize()
        return f.detach(), pooled, {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


if not args.skip_check:
    for (H, W, n, blocks) in [(16, 16, 300, 2), (16, 16, 1, 1), (16, 16, 3, 2), (9, 9, 203, 2), (8, 8, 70, 3),
                              (5, 7, 17, 2), (16, 16, 4096, 5), (9, 9, 8191, 5)]:
        for dt in (torch.float16, torch.bfloat16):
            m = model(blocks)
            obs = obs_(n, H, W)
            dms = dmasks(blocks, n)
            fa, pa, ga = run(m, obs, dt, dms, 2)
            fb, pb, gb = run(m, obs, dt, dms, 1)
            fc, pc, _ = run(m, obs, dt, dms, 2, grad=False)
            worst = max(gb, key=lambda k: rel(ga[k], gb[k]))
            print(f"{H}x{W} n={n} blocks={blocks} {str(dt)[6:]}: features rel {rel(fa, fb):.2e} "
                  f"max {(fa.float() - fb.float()).abs().max().item():.2e}; pooled rel {rel(pa, pb):.2e}; "
                  f"pooled vs mean {rel(pa, fa.float().mean(1)):.2e}; no-grad == saving: {torch.equal(fc, fa)} "
                  f"pooled {torch.equal(pc, pa)}; worst grad {worst} rel {rel(ga[worst], gb[worst]):.2e}", flush=True)

n = args.time_n
m = model(5)
obs = obs_(n, 16, 16)
dms = dmasks(5, n)
df = torch.randn(n, 256, 96, device=dev).to(torch.float16)


def timeit(variant):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    tf = tb = tn = 0.0
    with F.kernel_variant(F.VARIANT_TRUNK_FWD, variant):
        for it in range(args.iters + 2):
            m.zero_grad(set_to_none=True)
            ev[0].record()
            f = F.fused_features(m, obs, torch.float16, dmasks=dms)
            ev[1].record()
            f.backward(df)
            ev[2].record()
            del f
            with torch.no_grad():
                F.fused_features(m, obs, torch.float16, dmasks=dms)
            ev[3].record()
            torch.cuda.synchronize()
            if it >= 2:
                tf += ev[0].elapsed_time(ev[1])
                tb += ev[1].elapsed_time(ev[2])
                tn += ev[2].elapsed_time(ev[3])
    k = args.iters
    return tf / k, tb / k, tn / k


for r in range(3):
    for v in (0, 1, 2):
        a, b, c = timeit(v)
        print(f"round {r} variant {v} ({['default', 'fwd2', 'pp'][v]}): training fwd {a:.2f} ms, backward {b:.2f} ms, "
              f"no-grad fwd {c:.2f} ms (n={n}, incl. stem + obs encode)", flush=True)

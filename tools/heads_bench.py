"""Time mc_heads_bwd (k_heads_bwd + k_heads_reduce) at each BASELINE config's per-GPU PPO minibatch
and check it is deterministic (two launches bitwise equal).
    python tools/heads_bench.py [--iters 20]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minesweeper-ppo_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
import torch  # noqa: E402
from ms_amd import _lib as L  # noqa: E402
from ms_amd import fused  # noqa: E402

dev = torch.device("cuda")
C = 96
dt = torch.float16
fused._heads_bind()
st = L.stream_ptr(dev)
for n, P in ((32768, 256), (65536, 81), (8192, 480)):
    M = n * P
    torch.manual_seed(0)
    f = (torch.randn(n, P, C, device=dev) * 0.5).to(dt)
    w1 = (torch.randn(192, C, device=dev) * 0.1).to(dt)
    b1, w2 = torch.randn(192, device=dev) * 0.1, torch.randn(192, device=dev) * 0.1
    dlp, dlm = torch.randn(n, P, device=dev), torch.randn(n, P, device=dev)
    gadd = torch.randn(n, C, device=dev) / P
    nws = int(fused._hbws(M))
    work = torch.empty(nws, device=dev)

    def run():
        df = torch.empty_like(f)
        dw1, db1, dw2 = torch.empty(192, C, device=dev), torch.empty(192, device=dev), torch.empty(192, device=dev)
        fused._check(fused._hb(L.ptr(f), L.ptr(dlp), L.ptr(dlm), L.ptr(w1), None, L.ptr(b1), L.ptr(w2), L.ptr(gadd),
                               P, L.ptr(df), L.ptr(dw1), L.ptr(db1), L.ptr(dw2), L.ptr(work), nws, M, 1, st))
        return df, dw1, db1, dw2

    a = run()
    b = run()
    det = all(torch.equal(x, y) for x, y in zip(a, b))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.iters * 1e3
    gb = (2 * M * C * 2 + 2 * M * 4) / 1e9
    print(f"n={n} P={P}: {ms:.3f} ms (incl. k_heads_reduce), algorithmic {gb:.2f} GB -> {gb / ms:.2f} TB/s, "
          f"deterministic={det}", flush=True)

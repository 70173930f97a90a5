"""Timing of the value head's MLP (96 -> 256 -> 256 -> 1 on N pooled rows, cnn_residual.py:97-102)
forward + backward under fp16 autocast against alternative formulations (same process)."""
import sys
import time

import torch
import torch.nn.functional as F

N = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
dev = torch.device("cuda")
torch.manual_seed(0)
lin = [torch.nn.Linear(96, 256), torch.nn.Linear(256, 256), torch.nn.Linear(256, 1)]
lin = [m.to(dev) for m in lin]
x0 = torch.randn(N, 96, device=dev)


def mlp(x):
    return lin[2](F.relu(lin[1](F.relu(lin[0](x))))).squeeze(-1)


def run(name, fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    print(f"{name:40s} {(time.perf_counter() - t) / iters * 1e6:8.1f} us", flush=True)


def amp16():
    x = x0.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.float16):
        v = mlp(x)
    v.float().sum().backward()


def f32():
    x = x0.clone().requires_grad_(True)
    v = mlp(x)
    v.sum().backward()


def amp_bf16():
    x = x0.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        v = mlp(x)
    v.float().sum().backward()


def amp16_fwd():
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        mlp(x0)


def f32_fwd():
    with torch.no_grad():
        mlp(x0)


for lib in ["default", "cublas", "cublaslt"]:
    if lib != "default":
        torch.backends.cuda.preferred_blas_library(lib)
    print("blas:", torch.backends.cuda.preferred_blas_library())
    for name, fn in [("fp16 autocast fwd+bwd", amp16), ("fp32 fwd+bwd", f32), ("bf16 autocast fwd+bwd", amp_bf16),
                     ("fp16 autocast fwd (no grad)", amp16_fwd), ("fp32 fwd (no grad)", f32_fwd)]:
        run(name, fn)


# hand-written forward / backward (16-bit GEMMs forward and for the data gradients, f32
# split-K batched GEMMs for the weight gradients)
S = 32
W16 = [m.weight.detach().half() for m in lin]
B16 = [m.bias.detach().half() for m in lin]


def manual():
    x = x0.half()
    a1 = torch.addmm(B16[0], x, W16[0].t())
    h1 = torch.relu(a1)
    a2 = torch.addmm(B16[1], h1, W16[1].t())
    h2 = torch.relu(a2)
    v = torch.addmm(B16[2], h2, W16[2].t())
    dv = torch.ones_like(v)  # d(sum)/dv
    dh2 = (dv * W16[2]) * (a2 > 0)
    dw3 = (dv.float() * h2.float()).sum(0)
    dh1 = (dh2 @ W16[1]) * (a1 > 0)
    n = x.shape[0]
    dw2 = torch.bmm(dh2.float().view(S, n // S, -1).transpose(1, 2), h1.float().view(S, n // S, -1)).sum(0)
    dw1 = torch.bmm(dh1.float().view(S, n // S, -1).transpose(1, 2), x.float().view(S, n // S, -1)).sum(0)
    dx = dh1 @ W16[0]
    return dw1, dw2, dw3, dh2.float().sum(0), dh1.float().sum(0), dx


torch.backends.cuda.preferred_blas_library("cublaslt")
run("manual fwd+bwd (split-K f32 weight grads)", manual)

"""Per-tensor gradient error of one ppo_update on the shipped model against the reference's
fp32 CPU gradients (tests/golden/ppo_full_16x16.npz), for several device paths:
fp32 (MIOpen), fp32 with MIOpen disabled (native im2col GEMM), PyTorch bf16 autocast,
fused bf16. Diagnostic only (tools/)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "minesweeper-ppo_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

from conftest import golden  # noqa: E402
from test_parity_gpu import _batch, _full_train, _record_grads, _rel  # noqa: E402


def run(mode, dev):
    from ms_amd.ppo import FlatGrads, PPOConfig, ppo_update
    torch.set_float32_matmul_precision("highest")
    torch.backends.cudnn.enabled = mode != "fp32-nocudnn"
    z, m = _full_train(dev)
    m.fused = mode == "fused-bf16"
    opt = torch.optim.AdamW(m.parameters(), lr=3e-4)
    grads = _record_grads(m, opt)
    amp = torch.bfloat16 if "bf16" in mode else None
    ppo_update(m, opt, _batch(z, dev), PPOConfig(ent_coef=0.003, aux_mine_weight=0.05, aux_mine_calib_weight=0.01),
               scaler=None, amp_dtype=amp, flat_grads=FlatGrads(m.parameters()))
    torch.backends.cudnn.enabled = True
    return z, grads


def main():
    """python tools/grad_diag.py MODE [MODE ...]: per-tensor rel. L2 error vs the float64 truth,
    next to the reference's own fp32 error (run one process per MIOpen env setting)."""
    dev = torch.device("cuda:0")
    modes = sys.argv[1:] or ["fp32", "fp32-nocudnn", "torch-bf16", "fused-bf16"]
    res = {}
    for mode in modes:
        z, g = run(mode, dev)
        res[mode] = g
    names = list(res[modes[0]])
    tag = os.environ.get("DIAG_TAG", "")
    print(f"{tag} {'tensor':38s} {'ref-fp32':>10s} " + " ".join(f"{m:>13s}" for m in res))
    worst = {m: 0.0 for m in res}
    for k in names:
        t = z["grad64::" + k]
        ref = _rel(z["grad::" + k], t)
        row = [_rel(res[m][k], t) for m in res]
        if k != "policy_head.2.bias":
            for m, e in zip(res, row):
                worst[m] = max(worst[m], e / max(ref, 1e-6))
        print(f"{tag} {k:38s} {ref:10.3e} " + " ".join(f"{e:13.3e}" for e in row))
    print(tag, "worst error / reference fp32 error:", {m: round(v, 2) for m, v in worst.items()})


if __name__ == "__main__":
    main()

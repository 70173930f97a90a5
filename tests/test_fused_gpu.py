"""Fused conv3x3 + GroupNorm + residual + ReLU + dropout MFMA kernel vs a
PyTorch fp32 reference of the same op on the same bf16-rounded inputs.
Tolerance: |d| <= 2e-2 + 2e-2*|ref| (bf16 output rounding is 2^-8 relative)."""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(x, w, b, g, be, H, W, res=None, dmask=None):
    n, p, cin = x.shape
    xin = x.float().view(n, H, W, cin).permute(0, 3, 1, 2)
    wf = w.to(torch.bfloat16).float()
    y = F.conv2d(xin, wf[:, :cin] if wf.shape[1] >= cin else wf, b, padding=1)
    z = F.group_norm(y, 6, g, be, eps=1e-5)
    if res is not None:
        z = z + res.float().view(n, H, W, 96).permute(0, 3, 1, 2)
    z = torch.relu(z)
    if dmask is not None:
        z = z * dmask[:, :, None, None]
    to_nhwc = lambda t: t.permute(0, 2, 3, 1).reshape(n, p, 96)  # noqa: E731
    y = y.contiguous()
    mean = y.reshape(n, 6, -1).mean(-1)
    rstd = torch.rsqrt(y.reshape(n, 6, -1).var(-1, unbiased=False) + 1e-5)
    return to_nhwc(z), to_nhwc(y), torch.stack([mean, rstd], -1)


@pytest.mark.parametrize("H,W,cin,n", [(16, 16, 96, 300), (16, 16, 16, 37), (9, 9, 96, 70), (30, 16, 96, 20),
                                       (16, 30, 96, 9), (5, 7, 16, 3)])
@pytest.mark.parametrize("with_res", [False, True])
def test_conv_gn_fwd_matches_torch(gpu, H, W, cin, n, with_res):
    from ms_amd.fused import conv_gn_fwd, prep_weight
    torch.manual_seed(0)
    P = H * W
    x = (torch.randn(n, P, cin, device=gpu) * (0.5 if cin == 96 else 1.0)).to(torch.bfloat16)
    if cin == 16:
        x[:, :, 10:] = 0  # stem: 10 obs planes zero-padded to 16
    w = torch.randn(96, cin, 3, 3, device=gpu) * (1.0 / (3 * cin ** 0.5))
    b, g, be = torch.randn(96, device=gpu) * 0.1, 1 + 0.1 * torch.randn(96, device=gpu), 0.1 * torch.randn(96, device=gpu)
    res = torch.randn(n, P, 96, device=gpu).to(torch.bfloat16) if with_res else None
    dmask = ((torch.rand(n, 96, device=gpu) > 0.05).float() / 0.95) if not with_res else None
    out, y, st = conv_gn_fwd(x, prep_weight(w, cin), b, g, be, H, W, res=res, dmask=dmask)
    ro, ry, rst = _ref(x, w, b, g, be, H, W, res, dmask)
    torch.testing.assert_close(y.float(), ry, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(st, rst, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(out.float(), ro, atol=3e-2, rtol=2e-2)

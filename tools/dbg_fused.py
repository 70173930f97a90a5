import sys, torch
sys.path[:0] = ['/root/repo/minesweeper-ppo_amd', '/root/repo/tests', '/root/repo']
import os; sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/tests")
from test_fused_gpu import _ref
from ms_amd.fused import conv_gn_fwd, prep_weight
gpu = torch.device("cuda")
torch.manual_seed(0)
H, W, cin, n = 16, 16, 96, 4
P = H * W
x = (torch.randn(n, P, cin, device=gpu) * 0.5).to(torch.bfloat16)
w = torch.randn(96, cin, 3, 3, device=gpu) * (1.0 / (3 * cin ** 0.5))
b, g, be = torch.randn(96, device=gpu) * 0.1, 1 + 0.1 * torch.randn(96, device=gpu), 0.1 * torch.randn(96, device=gpu)
out, y, st = conv_gn_fwd(x, prep_weight(w, cin), b, g, be, H, W)
ro, ry, rst = _ref(x, w, b, g, be, H, W)
torch.set_printoptions(precision=5, sci_mode=False, linewidth=200)
print("kernel stats", st[:2])
print("ref stats", rst[:2])
yk = y.float().view(n, P, 6, 16)
print("kernel mean from ysave", yk.mean((1, 3))[:2], "var", yk.var((1,3), unbiased=False)[:2])
print("out maxdiff", (out.float() - ro).abs().max().item())

import torch, torch.nn.functional as F
for n in (37, 70, 128, 256, 1000):
    torch.manual_seed(0)
    y = torch.randn(n, 96, 16, 16, device="cuda", requires_grad=True)
    g = (1 + 0.1 * torch.randn(96, device="cuda")).requires_grad_(True)
    b = torch.zeros(96, device="cuda", requires_grad=True)
    z = F.group_norm(y, 6, g, b, eps=1e-5)
    dz = torch.randn_like(z)
    z.backward(dz)
    yh = (z - b[None, :, None, None]) / g[None, :, None, None]
    db = dz.sum((0, 2, 3)); dg = (dz * yh).sum((0, 2, 3))
    rel = lambda a, r: ((a - r).norm() / r.norm()).item()
    # CPU reference
    yc = y.detach().cpu().requires_grad_(True); gc = g.detach().cpu().requires_grad_(True); bc = b.detach().cpu().requires_grad_(True)
    F.group_norm(yc, 6, gc, bc, eps=1e-5).backward(dz.cpu())
    print(n, "gpu dbeta vs explicit", rel(b.grad, db), "dgamma", rel(g.grad, dg), "| cpu dbeta", rel(bc.grad, db.cpu()), "dgamma", rel(gc.grad, dg.cpu()), "| dy gpu vs cpu", rel(y.grad.cpu(), yc.grad))

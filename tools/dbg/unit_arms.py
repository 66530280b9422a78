"""tests/test_gpu_box.py::test_bn_prologue_fusion_bitwise (4-wave arm) repeated with fresh tuning:
prints the tuned plan and which results differ between the fused and unfused arms."""
import copy
import sys
import torch
sys.path.insert(0, ".")
from mil_nce_howto100m_amd.models.s3dg import STConv3D
from mil_nce_howto100m_amd.ops import hip_ops as h

DEV = "cuda"
shape, cin, cmid, k = (2, 8, 50, 50), 64, 192, (3, 3, 3)
torch.manual_seed(5)
unit = STConv3D(cin, cmid, list(k), padding=1, separable=True).cuda().train()
x = torch.randn(*shape, cin, device=DEV).to(torch.bfloat16)
g = torch.randn(*shape, cmid, device=DEV).to(torch.bfloat16)
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    h._PLANS.clear()
    res = {}
    for fuse in (False, True):
        h._PRO_FUSE = h._BNBWD_FUSE = fuse
        u = copy.deepcopy(unit)
        xi = x.clone().requires_grad_(True)
        out = u(xi)
        plan = h.conv_plan(tuple(shape) + (cmid,), (cmid, cmid, k[0], 1, 1), (1, 1, 1), (1, 0, 0))
        plan.impl = 16
        plan1 = h.conv_plan(tuple(shape) + (cin,), (cmid, cin, 1, k[1], k[2]), (1, 1, 1), (0, 1, 1))
        plan1.d_impl = 17
        xi.grad = None
        u.zero_grad()
        out = u(xi)
        out.backward(g)
        torch.cuda.synchronize()
        cur = {"out": out.detach().clone(), "dx": xi.grad.clone()}
        cur.update({n: p.grad.clone() for n, p in u.named_parameters()})
        res[fuse] = cur
    a, b = res[False], res[True]
    bad = [n for n in a if not torch.equal(a[n], b[n])]
    print(it, "temporal", plan.impl, plan.grid_m, plan.d_impl, plan.d_grid_m, "spatial", plan1.impl, plan1.grid_m,
          plan1.d_impl, plan1.d_grid_m, "w", plan.w_impl, plan1.w_impl, "differs:", bad, flush=True)

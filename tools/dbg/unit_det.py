"""Repeat a separable unit's forward/backward (as tests/test_gpu_box.py::test_bn_prologue_fusion_bitwise)
with fixed kernel choices and report which outputs change between repetitions."""
import copy
import sys
import torch
sys.path.insert(0, ".")
from mil_nce_howto100m_amd.models.s3dg import STConv3D
from mil_nce_howto100m_amd.ops import hip_ops as h

DEV = "cuda"
nw = int(sys.argv[1]) if len(sys.argv) > 1 else 4
fuse = int(sys.argv[2]) if len(sys.argv) > 2 else 1
shape, cin, cmid, k = (2, 8, 50, 50), 64, 192, (3, 3, 3)
torch.manual_seed(5)
unit = STConv3D(cin, cmid, list(k), padding=1, separable=True).cuda().train()
x = torch.randn(*shape, cin, device=DEV).to(torch.bfloat16)
g = torch.randn(*shape, cmid, device=DEV).to(torch.bfloat16)
h._PRO_FUSE = h._BNBWD_FUSE = bool(fuse)
u0 = copy.deepcopy(unit)
u0(x.clone().requires_grad_(True)).backward(g)  # tune everything
plan = h.conv_plan(tuple(shape) + (cmid,), (cmid, cmid, k[0], 1, 1), (1, 1, 1), (1, 0, 0))
plan1 = h.conv_plan(tuple(shape) + (cin,), (cmid, cin, 1, k[1], k[2]), (1, 1, 1), (0, 1, 1))
plan.impl = 16 if nw == 4 else 15
plan1.d_impl = 17 if nw == 4 else 15
print("temporal", plan.impl, plan.grid_m, plan.d_impl, plan.d_grid_m, "spatial", plan1.impl, plan1.grid_m,
      plan1.d_impl, plan1.d_grid_m, flush=True)
ref = None
for rep in range(6):
    u = copy.deepcopy(unit)
    xi = x.clone().requires_grad_(True)
    out = u(xi)
    out.backward(g)
    torch.cuda.synchronize()
    cur = {"out": out.detach().clone(), "dx": xi.grad.clone()}
    cur.update({n: p.grad.clone() for n, p in u.named_parameters()})
    if ref is None:
        ref = cur
    else:
        bad = [n for n in cur if not torch.equal(cur[n], ref[n])]
        print(rep, "differs:", bad, flush=True)

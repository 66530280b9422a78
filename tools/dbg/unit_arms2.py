"""unit_arms.py with the raw conv outputs / dgrad outputs of each arm recorded (monkeypatched hip_ops)."""
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
rec = []
orig_fwd, orig_dg, orig_dgb = h.conv_forward_raw, h.conv_dgrad, h.conv_dgrad_bnbwd


def fwd(x, wp, plan, stats, pro=None, shift=None):
    y = orig_fwd(x, wp, plan, stats, pro, shift)
    rec.append(("fwd", plan.k, plan.impl, plan.grid_m, y.clone(), None if shift is None else shift.clone()))
    return y


def dg(dy, wd, plan, producer_bn=None):
    dx = orig_dg(dy, wd, plan, producer_bn)
    rec.append(("dgrad", plan.k, plan.d_impl, plan.d_grid_m, dx.clone(), dy.clone()))
    return dx


def dgb(dz, wd, plan, producer_bn, y, ss, coef, dy_out, impl=0, grid=0, dx=None):
    r = orig_dgb(dz, wd, plan, producer_bn, y, ss, coef, dy_out, impl, grid, dx)
    rec.append(("dgradbn", plan.k, impl or plan.d_impl, grid or plan.d_grid_m, r.clone(), dz.clone(), dy_out.clone(),
                coef.clone(), y.clone()))
    return r


h.conv_forward_raw, h.conv_dgrad, h.conv_dgrad_bnbwd = fwd, dg, dgb
res = {}
for fuse in (False, True):
    h._PRO_FUSE = h._BNBWD_FUSE = fuse
    u = copy.deepcopy(unit)
    xi = x.clone().requires_grad_(True)
    out = u(xi)
    plan = h.conv_plan(tuple(shape) + (cmid,), (cmid, cmid, k[0], 1, 1), (1, 1, 1), (1, 0, 0))
    plan.impl = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    plan1 = h.conv_plan(tuple(shape) + (cin,), (cmid, cin, 1, k[1], k[2]), (1, 1, 1), (0, 1, 1))
    plan1.d_impl = int(sys.argv[2]) if len(sys.argv) > 2 else 17
    xi.grad = None
    u.zero_grad()
    rec.clear()
    out = u(xi)
    out.backward(g)
    torch.cuda.synchronize()
    res[fuse] = (list(rec), out.detach().clone(), xi.grad.clone())
    print("arm", fuse, [(r[0], r[1], r[2], r[3]) for r in rec], flush=True)
ra, rb = res[False][0], res[True][0]
for a, b in zip(ra, rb):
    diffs = [(i, torch.equal(ta, tb)) for i, (ta, tb) in enumerate(zip(a[4:], b[4:])) if torch.is_tensor(ta) and torch.is_tensor(tb) and ta.shape == tb.shape]
    print(a[0], a[1], a[2], "vs", b[0], b[1], b[2], diffs, flush=True)
print("out equal", torch.equal(res[False][1], res[True][1]), "dx equal", torch.equal(res[False][2], res[True][2]))

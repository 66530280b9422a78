"""Diagnose the pre-BN shift on the conv -> conv -> pool chain of test_fused_bn_backward_partials:
gradients against an fp32 ATen reference with a nonzero running mean, shift on / off, and with
the second conv's input applied lazily or materialised."""
import copy
import sys

import torch
import torch.nn as nn

sys.path.insert(0, ".")
from mil_nce_howto100m_amd.ops import aten  # noqa: E402
from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


torch.manual_seed(11)
DEV = "cuda"
B, T, H, W, c0, c1, c2 = 2, 4, 6, 6, 32, 48, 64
x = torch.randn(B, T, H, W, c0, device=DEV).to(torch.bfloat16)
convs = [nn.Conv3d(c0, c1, (1, 3, 3), 1, (0, 1, 1), bias=False).to(DEV),
         nn.Conv3d(c1, c2, (3, 1, 1), 1, (1, 0, 0), bias=False).to(DEV)]
bns = [nn.BatchNorm3d(c1).to(DEV), nn.BatchNorm3d(c2).to(DEV)]
with torch.no_grad():
    for b in bns:
        b.running_mean.uniform_(-0.3, 0.3)
g = None


def run(hip, materialize, shift, one_only=False):
    global g
    h._BN_SHIFT = shift
    bn = copy.deepcopy(bns)
    ws = [c.weight.detach().to(torch.bfloat16).float().clone().requires_grad_(True) for c in convs]
    xi = (x if hip else x.float()).clone().requires_grad_(True)
    if hip:
        z = h.conv_bn_relu(xi, ws[0], bn[0], (1, 1, 1), (0, 1, 1), True)
        if materialize:
            z = h._materialize(z)
        z1 = z
        z = h.conv_bn_relu(z, ws[1], bn[1], (1, 1, 1), (1, 0, 0), True)
        z = h.maxpool3d(z, (1, 3, 3), (1, 2, 2), True)
    else:
        z1 = z = aten.conv_bn_relu(xi, ws[0], bn[0], (1, 1, 1), (0, 1, 1), True)
        z = aten.conv_bn_relu(z, ws[1], bn[1], (1, 1, 1), (1, 0, 0), True)
        z = aten.maxpool_tf_same(z, (1, 3, 3), (1, 2, 2))
    if g is None:
        torch.manual_seed(12)
        g = torch.randn(z.shape, device=DEV)
    z.backward(g.to(z.dtype))
    z1v = h._materialize(z1) if hip and h._is_lazy(z1) else z1
    return [z.detach(), z1v.detach(), xi.grad] + [w.grad for w in ws] + [p.grad for b in bn for p in b.parameters()] \
        + [b.running_mean for b in bn]


ref = run(False, False, False)
names = ["out", "z1", "dx", "dw1", "dw2", "dg1", "db1", "dg2", "db2", "rm1", "rm2"]
for mat in (False,):
    for shift in (False, True):
        r = run(True, mat, shift)
        print(f"materialize={mat!s:5s} shift={shift!s:5s}", " ".join(f"{n} {rel(a, b):.4f}" for n, a, b in zip(names, r, ref)))

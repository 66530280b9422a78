"""Full-model gradient error vs an fp64 CPU oracle (8 x 64^2, batch 4, eval-mode BN as in
tests/test_gpu_gradcache.py) with the 4-wave box variants allowed / forced off: worst layers."""
import copy
import sys
import torch
sys.path.insert(0, ".")
from mil_nce_howto100m_amd.models import S3D
from mil_nce_howto100m_amd.ops import hip_ops as h

torch.manual_seed(0)
m0 = S3D(512).cuda().eval()
ref = copy.deepcopy(m0).cpu().double().eval()
v = torch.randint(0, 256, (4, 3, 8, 64, 64), dtype=torch.uint8)
t = torch.randint(0, 66250, (8, 20))
gv = torch.randn(4, 512, dtype=torch.float64)
gt = torch.randn(8, 512, dtype=torch.float64)


def run(model, vid, txt):
    ve, te = model(vid, txt)
    ((ve.double() * gv.to(ve.device)).sum() + (te.double() * gt.to(te.device)).sum()).backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().double().cpu() for n, p in model.named_parameters() if p.grad is not None}


gr = run(ref, v.double() / 255.0, t)
rel = lambda a, b: ((a - b).norm() / (b.norm() + 1e-30)).item()
flat_r = torch.cat([gr[n].flatten() for n in gr])
for box4 in (True, False, True):
    h._BOX4 = box4
    h._PLANS.clear()
    outs = []
    for rep in range(2):
        m = copy.deepcopy(m0)
        outs.append(run(m, v.cuda(), t.cuda()))
    g = outs[1]
    flat = torch.cat([g[n].flatten() for n in gr])
    errs = sorted(((rel(g[n], gr[n]), n) for n in gr), reverse=True)
    print(f"BOX4={box4}: whole-flat rel {rel(flat, flat_r):.4f}; worst:", flush=True)
    for e, n in errs[:8]:
        print(f"   {e:.4f} {n}")
    print("   4-wave kernels in plans:", sorted({(k[0][1:], p.impl, p.d_impl) for k, p in h._PLANS.items()
                                                   if p.impl in (16, 17) or p.d_impl in (16, 17)})[:12], flush=True)

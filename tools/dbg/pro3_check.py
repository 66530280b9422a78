"""Determinism / equality of the PRO 3 (BN-backward prologue) box dgrad: 8-wave vs 4-wave variants."""
import sys
import torch
sys.path.insert(0, ".")
from mil_nce_howto100m_amd.ops import hip_ops as h

DEV = "cuda"
torch.manual_seed(3)
B, T, H, W, cx, C = 2, 8, 50, 50, 64, 192   # dgrad: dz [.., C] -> dx [.., cx]
k, p = (1, 3, 3), (0, 1, 1)
plan = h.conv_plan((B, T, H, W, cx), (C, cx, *k), (1, 1, 1), p)
w = torch.randn(C, cx, *k, device=DEV) * 0.05
wd = h._pack(w, plan, 1)
dz = torch.randn(B, T, H, W, C, device=DEV).to(torch.bfloat16)
y = torch.randn(B, T, H, W, C, device=DEV).to(torch.bfloat16)
ss = torch.cat([torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5,
                torch.randn(C, device=DEV), torch.randn(C, device=DEV) * 0.2])
coef = torch.randn(3 * C, device=DEV) * 0.1
res = {}
for impl in (15, 17, 14, 16):
    grid = h._grid_for(plan.M, plan.d_Npad, h._box_eff_bn(impl, plan.d_bn), 2 if impl >= 16 else 1)
    outs = []
    for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
        dy = torch.zeros_like(y)
        dx = h.conv_dgrad_bnbwd(dz, wd, plan, None, y, ss, coef, dy, impl, grid)
        torch.cuda.synchronize()
        outs.append((dx.clone(), dy.clone()))
    same = [torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1]) for o in outs]
    res[impl] = outs[0]
    print(impl, "grid", grid, "deterministic", all(same), same)
for a, b in ((15, 17), (14, 16)):
    dxa, dya = res[a]
    dxb, dyb = res[b]
    bad = (dxa != dxb).nonzero()
    print(a, b, "dx equal", torch.equal(dxa, dxb), "dy equal", torch.equal(dya, dyb), "ndiff", bad.shape[0],
          bad[:8].tolist())

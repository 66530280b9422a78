"""Determinism and 8-wave / 4-wave equality of the box kernels on the conv_2c shapes
(forward with EPI 1 and PRO 2 / dgrad with EPI 2), repeated launches."""
import sys
import torch
sys.path.insert(0, ".")
from mil_nce_howto100m_amd.ops import hip_ops as h

DEV = "cuda"
REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
torch.manual_seed(3)
B, T, H, W = 2, 8, 50, 50


def check(cin, cout, k, p, pairs):
    plan = h.conv_plan((B, T, H, W, cin), (cout, cin, *k), (1, 1, 1), p)
    w = torch.randn(cout, cin, *k, device=DEV) * 0.05
    wp, wd = h._pack(w, plan, 0), h._pack(w, plan, 1)
    x = torch.randn(B, T, H, W, cin, device=DEV).to(torch.bfloat16)
    dy = torch.randn(B, T, H, W, cout, device=DEV).to(torch.bfloat16)
    ss = torch.cat([torch.randn(cin, device=DEV) * 0.1, torch.rand(cin, device=DEV) + 0.5,
                    torch.randn(cin, device=DEV), torch.randn(cin, device=DEV) * 0.2])
    stats = torch.empty((h._stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad,), device=DEV)
    res = {}
    for impl in sorted({i for pr in pairs for i in pr}):
        outs = []
        for rep in range(REPS):
            plan.impl = plan.d_impl = impl
            wgs = 2 if impl >= 16 else 1
            plan.grid_m = h._grid_for(plan.M, plan.Npad, h._box_eff_bn(impl, plan.bn), wgs)
            plan.d_grid_m = h._grid_for(plan.M, plan.d_Npad, h._box_eff_bn(impl, plan.d_bn), wgs)
            try:
                y = h.conv_forward_raw(x, wp, plan, stats)
                st = stats[:plan.grid_m * 2 * plan.Npad].view(plan.grid_m, 2, plan.Npad).double().sum(0)
                dx = h.conv_dgrad(dy, wd, plan, (x, ss, cin))
                part, nparts, ps = h.take_bn_partials(dx)
                pst = part[:nparts * 2 * ps].view(nparts, 2, ps).double().sum(0)
            except h.UnsupportedVariant:
                print(cin, cout, k, impl, "unsupported")
                break
            torch.cuda.synchronize()
            outs.append((y.clone(), dx.clone(), st, pst))
        if not outs:
            continue
        det = [torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1]) for o in outs]
        res[impl] = outs[0]
        print(cin, cout, k, impl, "deterministic", all(det), det, flush=True)
    for a, b in pairs:
        if a in res and b in res:
            print(cin, cout, k, a, b, "y equal", torch.equal(res[a][0], res[b][0]), "dx equal",
                  torch.equal(res[a][1], res[b][1]),
                  "stats maxrel %.2e" % ((res[a][2] - res[b][2]).abs().max() / res[a][2].abs().max()).item(),
                  "partials maxrel %.2e" % ((res[a][3] - res[b][3]).abs().max() / res[a][3].abs().max()).item(),
                  flush=True)


check(192, 192, (3, 1, 1), (1, 0, 0), [(15, 17), (14, 16)])
check(64, 192, (1, 3, 3), (0, 1, 1), [(15, 17), (14, 16)])
check(128, 128, (3, 1, 1), (1, 0, 0), [(15, 17), (14, 16)])

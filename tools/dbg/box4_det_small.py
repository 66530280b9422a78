"""Run-to-run determinism of the 4-wave box variants (fwd EPI 1 / dgrad EPI 2 / PRO 3 dgrad) on the
layer shapes of an 8 x 64^2 clip batch of 4."""
import sys
import torch
sys.path.insert(0, ".")
from mil_nce_howto100m_amd.ops import hip_ops as h

DEV = "cuda"
torch.manual_seed(3)
SHAPES = [((4, 8, 8), 16, 32, (1, 3, 3)), ((4, 8, 8), 32, 32, (3, 1, 1)), ((4, 8, 8), 96, 128, (1, 3, 3)),
          ((4, 8, 8), 128, 128, (3, 1, 1)), ((4, 16, 16), 64, 192, (1, 3, 3)), ((4, 16, 16), 192, 192, (3, 1, 1)),
          ((4, 8, 8), 128, 192, (1, 3, 3)), ((4, 8, 8), 192, 192, (3, 1, 1)), ((4, 8, 8), 32, 96, (1, 3, 3)),
          ((4, 8, 8), 96, 96, (3, 1, 1))]
B = 4
bad = 0
for (T, H, W), cin, cout, k in SHAPES:
    pad = tuple(kk // 2 for kk in k)
    plan = h.conv_plan((B, T, H, W, cin), (cout, cin, *k), (1, 1, 1), pad)
    w = torch.randn(cout, cin, *k, device=DEV) * 0.05
    wp, wd = h._pack(w, plan, 0), h._pack(w, plan, 1)
    x = torch.randn(B, T, H, W, cin, device=DEV).to(torch.bfloat16)
    dy = torch.randn(B, T, H, W, cout, device=DEV).to(torch.bfloat16)
    ss = torch.cat([torch.randn(cin, device=DEV) * 0.1, torch.rand(cin, device=DEV) + 0.5,
                    torch.randn(cin, device=DEV), torch.randn(cin, device=DEV) * 0.2])
    sso = torch.cat([torch.randn(cout, device=DEV) * 0.1, torch.rand(cout, device=DEV) + 0.5,
                     torch.randn(cout, device=DEV), torch.randn(cout, device=DEV) * 0.2])
    coef = torch.randn(3 * cout, device=DEV) * 0.1
    yo = torch.randn(B, T, H, W, cout, device=DEV).to(torch.bfloat16)
    stats = torch.empty((h._stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad,), device=DEV)
    for impl in (14, 15, 16, 17):
        geo = h._box_geo(plan)
        fok, dok = h._box_ok(plan.bn, cin, plan.Kpad, impl, geo), h._box_ok(plan.d_bn, cout, plan.d_Kpad, impl, geo)
        wgs = 2 if impl >= 16 else 1
        res = []
        for rep in range(4):
            out = []
            try:
                if fok:
                    plan.impl, plan.grid_m = impl, h._grid_for(plan.M, plan.Npad, h._box_eff_bn(impl, plan.bn), wgs)
                    y = h.conv_forward_raw(x, wp, plan, stats)
                    out += [y.clone(), stats[:plan.grid_m * 2 * plan.Npad].clone()]
                if dok:
                    plan.d_impl = impl
                    plan.d_grid_m = h._grid_for(plan.M, plan.d_Npad, h._box_eff_bn(impl, plan.d_bn), wgs)
                    dx = h.conv_dgrad(dy, wd, plan, (x, ss, cin))
                    part, nparts, ps = h.take_bn_partials(dx)
                    out += [dx.clone(), part[:nparts * 2 * ps].clone()]
                    if h._box_pro3_ok(impl, plan):
                        dyo = torch.zeros_like(yo)
                        dx2 = h.conv_dgrad_bnbwd(yo, wd, plan, (x, ss, cin), yo, sso, coef, dyo, impl, plan.d_grid_m)
                        part, nparts, ps = h.take_bn_partials(dx2)
                        out += [dx2.clone(), dyo.clone(), part[:nparts * 2 * ps].clone()]
            except h.UnsupportedVariant:
                out = None
            torch.cuda.synchronize()
            res.append(out)
        if res[0] is None or not res[0]:
            continue
        same = [all(torch.equal(a, b) for a, b in zip(r, res[0])) for r in res[1:]]
        which = [[i for i, (a, b) in enumerate(zip(r, res[0])) if not torch.equal(a, b)] for r in res[1:]]
        if not all(same):
            bad += 1
        print((T, H, W), cin, cout, k, impl, "fwd" if fok else "", "dgrad" if dok else "",
              "deterministic" if all(same) else f"NONDETERMINISTIC {which}", flush=True)
print("nondeterministic cases:", bad)

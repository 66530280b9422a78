"""Cold-cache correctness of box variants vs a warm run, over configurations (PRO 0 / 2, EPI 0 / 1)."""
import sys
import torch
sys.path.insert(0, ".")
from mil_nce_howto100m_amd.ops import hip_ops as h
from mil_nce_howto100m_amd.ops._lib import call, ptr, stream

DEV = "cuda"
flush = torch.empty((384 << 20) // 4, device=DEV)


def run(shape, ld, c0, cin, cout, k, p, impl, pro, epi, reps=6):
    torch.manual_seed(3)
    B, T, H, W = shape
    plan = h.conv_plan((B, T, H, W, cin), (cout, cin, *k), (1, 1, 1), p)
    if not h._box_ok(plan.bn, cin, plan.Kpad, impl, h._box_geo(plan)):
        return None
    w = torch.randn(cout, cin, *k, device=DEV) * 0.05
    wp = h._pack(w, plan, 0)
    full = torch.randn(B, T, H, W, ld, device=DEV).to(torch.bfloat16)
    yp = full[..., c0:]
    ss = torch.cat([torch.randn(cin, device=DEV) * 0.1, torch.rand(cin, device=DEV) + 0.5,
                    torch.rand(cin, device=DEV) + 0.5, torch.randn(cin, device=DEV) * 0.2])
    shift = torch.randn(cout, device=DEV) * 0.1
    grid = h._grid_for(plan.M, plan.Npad, h._box_eff_bn(impl, plan.bn), 2 if impl >= 16 else 1)
    outs = []
    for rep in range(reps):
        if rep % 2 == 0:
            flush.zero_()
        y = torch.full((B, T, H, W, cout), 3.0, dtype=torch.bfloat16, device=DEV)
        z = torch.empty((B, T, H, W, cin), dtype=torch.bfloat16, device=DEV)
        stats = torch.zeros(h._stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad, device=DEV) if epi else None
        try:
            if pro:
                call("milnce_conv_fwd_pro", ptr(yp), ld, ptr(wp), ptr(y), ptr(stats), ptr(shift) if epi else None,
                     ptr(ss), ptr(z) if pro == 2 else None,
                     B, T, H, W, cin, cout, *k, *p, plan.Kpad, plan.Npad, cout, plan.bn, grid, impl, stream())
            else:
                xin = yp.contiguous()
                call("milnce_conv_fwd", ptr(xin), 0, ptr(wp), ptr(y), ptr(stats), None, ptr(shift) if epi else None, 0,
                     B, T, H, W, cin, cout, *k, 1, 1, 1, *p, plan.Kpad, plan.Npad, cout, plan.bn, 64, grid, 0, impl,
                     stream())
        except h.UnsupportedVariant:
            return None
        torch.cuda.synchronize()
        outs.append(y)
    ref = outs[1]
    return [(o != ref).sum().item() for o in outs]


cases = [((4, 4, 8, 8), 176, 64, 96, 128, (1, 3, 3), (0, 1, 1)),
         ((8, 8, 25, 25), 96, 0, 96, 96, (1, 3, 3), (0, 1, 1)),
         ((8, 8, 25, 25), 64, 0, 64, 128, (1, 3, 3), (0, 1, 1)),
         ((8, 8, 25, 25), 128, 0, 128, 128, (1, 3, 3), (0, 1, 1)),
         ((8, 8, 25, 25), 192, 0, 192, 192, (3, 1, 1), (1, 0, 0)),
         ((8, 8, 50, 50), 64, 0, 64, 192, (1, 3, 3), (0, 1, 1))]
nbad = 0
for c in cases:
    for impl in (14, 15, 16, 17):
        for pro, epi in ((0, 0), (0, 1), (2, 1), (1, 0)):
            r = run(*c, impl, pro, epi, reps=8)
            if r is not None and any(r):
                nbad += 1
                print(c[0], c[3], c[4], c[5], "impl", impl, "pro", pro, "epi", epi, "mismatches", r, flush=True)
print("done; configurations with cold-cache mismatches:", nbad)

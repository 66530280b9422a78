"""PRO 2 (BN-ReLU prologue, z written) vs bn_relu_apply + PRO 0 for every box variant, repeated."""
import sys
import torch
sys.path.insert(0, ".")
from mil_nce_howto100m_amd.ops import hip_ops as h
from mil_nce_howto100m_amd.ops._lib import call, ptr, stream

DEV = "cuda"
torch.manual_seed(3)


def check(shape, cin, cout, k, p):
    B, T, H, W = shape
    plan = h.conv_plan((B, T, H, W, cin), (cout, cin, *k), (1, 1, 1), p)
    w = torch.randn(cout, cin, *k, device=DEV) * 0.05
    wp = h._pack(w, plan, 0)
    yp = torch.randn(B, T, H, W, cin, device=DEV).to(torch.bfloat16)
    ss = torch.cat([torch.randn(cin, device=DEV) * 0.1, torch.rand(cin, device=DEV) + 0.5,
                    torch.rand(cin, device=DEV) + 0.5, torch.randn(cin, device=DEV) * 0.2])
    rows = h._stats_rows(plan.M, plan.Npad, plan.bn)
    z0 = torch.empty_like(yp)
    call("milnce_bn_relu_apply", ptr(yp), cin, ptr(z0), cin, ptr(ss), cin, B, T * H * W, None, stream())
    for impl in h._BOX_IMPLS:
        if not h._box_ok(plan.bn, cin, plan.Kpad, impl, h._box_geo(plan)):
            continue
        grid = h._grid_for(plan.M, plan.Npad, h._box_eff_bn(impl, plan.bn), 2 if impl >= 16 else 1)
        outs = []
        for rep in range(4):
            for pro in (0, 1):
                y = torch.empty(B, T, H, W, cout, dtype=torch.bfloat16, device=DEV)
                stats = torch.zeros(rows * 2 * plan.Npad, device=DEV)
                z = torch.full_like(yp, 7.0)
                try:
                    if pro:
                        call("milnce_conv_fwd_pro", ptr(yp), cin, ptr(wp), ptr(y), ptr(stats), None, ptr(ss), ptr(z),
                             B, T, H, W, cin, cout, *k, *p, plan.Kpad, plan.Npad, cout, plan.bn, grid, impl, stream())
                    else:
                        call("milnce_conv_fwd", ptr(z0), 0, ptr(wp), ptr(y), ptr(stats), None, None, 0, B, T, H, W, cin,
                             cout, *k, 1, 1, 1, *p, plan.Kpad, plan.Npad, cout, plan.bn, 64, grid, 0, impl, stream())
                except h.UnsupportedVariant:
                    outs = None
                    break
                torch.cuda.synchronize()
                outs.append((pro, y, z, stats))
            if outs is None:
                break
        if outs is None:
            print(shape, cin, cout, k, impl, "unsupported")
            continue
        y0 = outs[0][1]
        ydiff = [(o[0], (o[1] != y0).sum().item()) for o in outs]
        zbad = [(o[2] != z0).sum().item() for o in outs if o[0] == 1]
        print(shape, cin, cout, k, impl, "grid", grid, "y mismatches (pro, n):", ydiff, "z mismatches:", zbad, flush=True)


check((2, 8, 50, 50), 192, 192, (3, 1, 1), (1, 0, 0))
check((2, 8, 50, 50), 64, 192, (1, 3, 3), (0, 1, 1))
check((2, 8, 25, 25), 128, 192, (1, 3, 3), (0, 1, 1))
check((2, 4, 13, 13), 160, 320, (3, 1, 1), (1, 0, 0))

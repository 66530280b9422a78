"""PRO 1 (BN-ReLU prologue, no z) with x a channel slice (x_ld > Cin), eval mode (no statistics):
run-to-run determinism per box variant, against the unfused reference."""
import sys
import torch
sys.path.insert(0, ".")
from mil_nce_howto100m_amd.ops import hip_ops as h
from mil_nce_howto100m_amd.ops._lib import call, ptr, stream

DEV = "cuda"
torch.manual_seed(3)


def check(shape, ld, c0, cin, cout, k, p, zmode=0, epi=0):
    B, T, H, W = shape
    plan = h.conv_plan((B, T, H, W, cin), (cout, cin, *k), (1, 1, 1), p)
    w = torch.randn(cout, cin, *k, device=DEV) * 0.05
    wp = h._pack(w, plan, 0)
    full = torch.randn(B, T, H, W, ld, device=DEV).to(torch.bfloat16)
    yp = full[..., c0:]  # slice start; rows of ld elements
    ss = torch.cat([torch.randn(cin, device=DEV) * 0.1, torch.rand(cin, device=DEV) + 0.5,
                    torch.rand(cin, device=DEV) + 0.5, torch.randn(cin, device=DEV) * 0.2])
    z0 = torch.empty(B, T, H, W, cin, dtype=torch.bfloat16, device=DEV)
    call("milnce_bn_relu_apply", ptr(yp), ld, ptr(z0), cin, ptr(ss), cin, B, T * H * W, None, stream())
    for impl in h._BOX_IMPLS:
        if not h._box_ok(plan.bn, cin, plan.Kpad, impl, h._box_geo(plan)):
            continue
        grid = h._grid_for(plan.M, plan.Npad, h._box_eff_bn(impl, plan.bn), 2 if impl >= 16 else 1)
        ys = []
        for rep in range(5):
            y = torch.full((B, T, H, W, cout), 3.0, dtype=torch.bfloat16, device=DEV)
            z = torch.full((B, T, H, W, cin), 5.0, dtype=torch.bfloat16, device=DEV) if zmode else None
            stats = torch.zeros(h._stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad, device=DEV) if epi else None
            try:
                call("milnce_conv_fwd_pro", ptr(yp), ld, ptr(wp), ptr(y), ptr(stats), None, ptr(ss), ptr(z),
                     B, T, H, W, cin, cout, *k, *p, plan.Kpad, plan.Npad, cout, plan.bn, grid, impl, stream())
            except h.UnsupportedVariant:
                ys = None
                break
            torch.cuda.synchronize()
            ys.append(y)
        if ys is None:
            print(shape, ld, cin, cout, k, impl, "unsupported")
            continue
        yref = torch.empty_like(ys[0])
        call("milnce_conv_fwd", ptr(z0), 0, ptr(wp), ptr(yref), None, None, None, 0, B, T, H, W, cin, cout, *k,
             1, 1, 1, *p, plan.Kpad, plan.Npad, cout, plan.bn, 64, grid, 0, impl, stream())
        torch.cuda.synchronize()
        nd = [(y != ys[0]).sum().item() for y in ys[1:]]
        print(shape, ld, cin, cout, k, impl, "grid", grid, "run-to-run mismatches", nd,
              "vs unfused", (ys[0] != yref).sum().item(), flush=True)


for zm, ep in ((1, 0), (1, 1), (0, 1)):
    print("== z written" if zm else "== no z", "stats" if ep else "no stats", flush=True)
    check((4, 4, 8, 8), 176, 64, 96, 128, (1, 3, 3), (0, 1, 1), zm, ep)
    check((4, 4, 8, 8), 128, 0, 128, 128, (3, 1, 1), (1, 0, 0), zm, ep)
    check((4, 4, 8, 8), 352, 128, 128, 192, (1, 3, 3), (0, 1, 1), zm, ep)
    check((4, 4, 8, 8), 96, 0, 96, 96, (3, 1, 1), (1, 0, 0), zm, ep)
    check((4, 4, 8, 8), 192, 0, 192, 192, (3, 1, 1), (1, 0, 0), zm, ep)

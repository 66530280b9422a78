#!/usr/bin/env python3
"""Time the box dgrads with the BN-backward prologue (PRO 3, hip_ops.conv_dgrad_bnbwd) per variant
at a flagship layer (default: conv_2c spatial, 1x3x3 64 -> 192 at 256 x 8 x 50 x 50): the 8-wave
(14 / 15) and 4-wave (16 / 17) box kernels on their persistent grids, cold-cache timing as in the
tuner. Variants that decline the shape (LDS / register budget) are listed as such.

    python tools/bnbwd_bench.py [--shape B T H W] [--cin 64] [--cout 192]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402

DEV = "cuda"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs=4, default=[256, 8, 50, 50])
    ap.add_argument("--cin", type=int, default=64)
    ap.add_argument("--cout", type=int, default=192)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    B, T, H, W = a.shape
    torch.manual_seed(0)
    x = torch.randn(B, T, H, W, a.cin, device=DEV).to(torch.bfloat16)
    w = torch.randn(a.cout, a.cin, 1, 3, 3, device=DEV) * 0.05
    plan = h.conv_plan(x.shape, w.shape, (1, 1, 1), (0, 1, 1))
    wd = h._pack(w, plan, 1)
    y = torch.randn(B, T, H, W, a.cout, device=DEV).to(torch.bfloat16)
    dz = torch.randn_like(y)
    C = a.cout
    ss = torch.cat([torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5,
                    torch.randn(C, device=DEV), torch.randn(C, device=DEV) * 0.2])
    coef = torch.cat([torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.01,
                      torch.randn(C, device=DEV) * 0.01])
    xss = torch.cat([torch.randn(a.cin, device=DEV) * 0.1, torch.rand(a.cin, device=DEV) + 0.5,
                     torch.randn(a.cin, device=DEV), torch.randn(a.cin, device=DEV) * 0.2])
    dy = torch.empty_like(y)
    md = B * T * H * W
    flush = torch.empty((384 << 20) // 4, device=DEV)
    geo = h._box_geo(plan)
    print(f"plan d_bn {plan.d_bn} d_Npad {plan.d_Npad} d_Kpad {plan.d_Kpad} M {md}", flush=True)
    for impl in (14, 15, 16, 17):
        if not h._box_ok(plan.d_bn, C, plan.d_Kpad, impl, geo) or not h._box_pro3_ok(impl, plan):
            print(f"impl {impl}: not a candidate", flush=True)
            continue
        for wgs in ((1, 2) if impl in (14, 15) else (2,)):
            grid = h._grid_for(md, plan.d_Npad, h._box_eff_bn(impl, plan.d_bn), wgs)
            try:
                h.conv_dgrad_bnbwd(dz, wd, plan, (x, xss, a.cin), y, ss, coef, dy, impl, grid)
            except h.UnsupportedVariant as e:
                print(f"impl {impl} wgs {wgs}: declined ({e})", flush=True)
                continue
            ts = []
            for _ in range(a.reps):
                flush.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                h.conv_dgrad_bnbwd(dz, wd, plan, (x, xss, a.cin), y, ss, coef, dy, impl, grid)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            print(f"impl {impl} wgs {wgs} grid {grid}: {ts[len(ts) // 2]:.3f} ms (min {ts[0]:.3f})", flush=True)


if __name__ == "__main__":
    main()

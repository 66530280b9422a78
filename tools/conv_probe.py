#!/usr/bin/env python3
"""Run one conv layer's forward / dgrad / wgrad kernels a few times (for rocprofv3 --pmc passes).

    python tools/conv_probe.py [--cin 64 --cout 192 --k 1 3 3 --t 8 --hw 50 --batch 256]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=64)
    ap.add_argument("--cout", type=int, default=192)
    ap.add_argument("--k", type=int, nargs=3, default=[1, 3, 3])
    ap.add_argument("--t", type=int, default=8)
    ap.add_argument("--hw", type=int, default=50)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    o = ap.parse_args()
    k = tuple(o.k)
    pad = tuple(kk // 2 for kk in k)
    x = torch.randn(o.batch, o.t, o.hw, o.hw, o.cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(o.cout, o.cin, *k, device="cuda") * 0.05
    plan = h.conv_plan(x.shape, w.shape, (1, 1, 1), pad)
    wp, wd = h._pack(w, plan, 0), h._pack(w, plan, 1)
    stats = torch.empty((h._stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad,), device="cuda")
    y = h.conv_forward_raw(x, wp, plan, stats)  # autotunes
    dy = torch.randn_like(y)
    h.conv_dgrad(dy, wd, plan)
    h.conv_wgrad(dy, x, plan)
    torch.cuda.synchronize()
    print(f"impl fwd {plan.impl} dgrad {plan.d_impl} wgrad {plan.w_impl}; tiles bn={plan.bn} bk={plan.bk} "
          f"wgrad {plan.w_tn}x{plan.w_tk} splits {plan.w_splits}")
    for _ in range(o.reps):
        h.conv_forward_raw(x, wp, plan, stats)
        h.conv_dgrad(dy, wd, plan)
        h.conv_wgrad(dy, x, plan)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Time every forward / dgrad kernel variant of one conv shape in isolation (csrc/conv.hip
launch_v3_impl ids), with the BN-statistics epilogue the training step uses.

    python tools/conv_impls.py [--cin 64 --cout 192 --k 1 3 3 --t 8 --hw 50 --batch 256 --impls 3 4 5 7]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402


FLUSH = None


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    if FLUSH is not None:  # cold caches before every launch, as inside the step (hip_ops._tune_local)
        tot = 0.0
        for _ in range(reps):
            FLUSH.zero_()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            tot += a.elapsed_time(b)
        return tot / reps
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=64)
    ap.add_argument("--cout", type=int, default=192)
    ap.add_argument("--k", type=int, nargs=3, default=[1, 3, 3])
    ap.add_argument("--t", type=int, default=8)
    ap.add_argument("--hw", type=int, default=50)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--impls", type=int, nargs="+", default=[3, 4, 5, 7])
    ap.add_argument("--producer", type=int, default=0,
                    help="1: dgrad with the producer-BN partials epilogue (as in the training step)")
    ap.add_argument("--cold", type=int, default=1, help="flush L2 / MALL before each timed launch")
    o = ap.parse_args()
    global FLUSH
    if o.cold:
        FLUSH = torch.empty((384 << 20) // 4, device="cuda")
    k = tuple(o.k)
    pad = tuple(kk // 2 for kk in k)
    x = torch.randn(o.batch, o.t, o.hw, o.hw, o.cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(o.cout, o.cin, *k, device="cuda") * 0.05
    plan = h.conv_plan(x.shape, w.shape, (1, 1, 1), pad)
    wp, wd = h._pack(w, plan, 0), h._pack(w, plan, 1)
    stats = torch.empty((h._stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad,), device="cuda")
    dy = torch.randn(plan.B, plan.To, plan.Ho, plan.Wo, o.cout, device="cuda").to(torch.bfloat16)
    fl = 2.0 * plan.M * plan.Cout * plan.Ktot
    prod = None
    if o.producer:  # the producer BN of x: y = x, arbitrary scale / shift
        ss = torch.cat([torch.zeros(o.cin, device="cuda"), torch.ones(o.cin, device="cuda"),
                        torch.ones(o.cin, device="cuda"), torch.zeros(o.cin, device="cuda")])
        prod = (x, ss, o.cin)
    print(f"{tuple(x.shape)} -> {o.cout} k{k}: fwd tile bn {plan.bn} bk {plan.bk}, dgrad tile bn {plan.d_bn} "
          f"bk {plan.d_bk}; {fl / 1e9:.0f} GFLOP", flush=True)
    g0, dg0 = plan.grid_m, plan.d_grid_m
    for impl in o.impls:
        plan.pin_f = plan.pin_d = impl
        # the 256-row variants hold one workgroup per CU: persistent grid of 1 per CU
        wide = impl in h._V4_WIDE_M
        md = plan.B * plan.T * plan.H * plan.W
        if impl in h._BOX4_IMPLS:  # 4-wave box workgroups: two per CU
            plan.grid_m = h._grid_for(plan.M, plan.Npad, h._box_eff_bn(impl, plan.bn), 2)
            plan.d_grid_m = h._grid_for(md, plan.d_Npad, h._box_eff_bn(impl, plan.d_bn), 2)
        else:
            plan.grid_m = h._grid_for(plan.M, plan.Npad, plan.bn, 1) if wide else g0
            plan.d_grid_m = h._grid_for(md, plan.d_Npad, plan.d_bn, 1) if wide else dg0
        try:
            tf = timeit(lambda: h.conv_forward_raw(x, wp, plan, stats))
            td = timeit(lambda: h.conv_dgrad(dy, wd, plan, prod))
        except Exception as e:  # variant not available for this tile
            print(f"impl {impl}: {e}")
            continue
        print(f"impl {impl}: fwd {tf:7.3f} ms {fl / tf / 1e9:6.0f} TF/s   dgrad {td:7.3f} ms {fl / td / 1e9:6.0f} TF/s",
              flush=True)


if __name__ == "__main__":
    main()

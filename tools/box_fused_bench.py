#!/usr/bin/env python3
"""Cold-cache timings of the box kernels' fused paths per variant (csrc/conv_box.hip): the forward
with the producer's BN-ReLU prologue (PRO 2, z written, BN statistics epilogue) and the dgrad with
the BN-backward prologue (PRO 3, dy written) and the producer-BN partials epilogue, as the training
step runs them.

    python tools/box_fused_bench.py --cin 64 --cout 192 --k 1 3 3 --t 8 --hw 50 --batch 256
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402
from mil_nce_howto100m_amd.ops._lib import call, ptr, stream  # noqa: E402


def timeit(fn, flush, reps=8):
    fn()
    torch.cuda.synchronize()
    tot = []
    for _ in range(reps):
        flush.zero_()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        tot.append(a.elapsed_time(b))
    return sorted(tot)[len(tot) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=64)
    ap.add_argument("--cout", type=int, default=192)
    ap.add_argument("--k", type=int, nargs=3, default=[1, 3, 3])
    ap.add_argument("--t", type=int, default=8)
    ap.add_argument("--hw", type=int, default=50)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--impls", type=int, nargs="+", default=[14, 15, 16, 17])
    o = ap.parse_args()
    dev = "cuda"
    flush = torch.empty((384 << 20) // 4, device=dev)
    k = tuple(o.k)
    pad = tuple(kk // 2 for kk in k)
    B, T, H, W, cin, cout = o.batch, o.t, o.hw, o.hw, o.cin, o.cout
    plan = h.conv_plan((B, T, H, W, cin), (cout, cin, *k), (1, 1, 1), pad)
    w = torch.randn(cout, cin, *k, device=dev) * 0.05
    wp, wd = h._pack(w, plan, 0), h._pack(w, plan, 1)
    yp = torch.randn(B, T, H, W, cin, device=dev).to(torch.bfloat16)  # the producer's raw output
    ssi = torch.cat([torch.zeros(cin, device=dev), torch.ones(cin, device=dev), torch.ones(cin, device=dev),
                     torch.zeros(cin, device=dev)])
    y = torch.empty(B, T, H, W, cout, dtype=torch.bfloat16, device=dev)
    z = torch.empty_like(yp)
    stats = torch.empty((h._stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad,), device=dev)
    # dgrad side: dz and y of this conv's BN ([cout]), coefficients, dy out; dx with the producer partials
    dz = torch.randn(B, T, H, W, cout, device=dev).to(torch.bfloat16)
    yo = torch.randn(B, T, H, W, cout, device=dev).to(torch.bfloat16)
    sso = torch.cat([torch.zeros(cout, device=dev), torch.ones(cout, device=dev), torch.ones(cout, device=dev),
                     torch.zeros(cout, device=dev)])
    coef = torch.randn(3 * cout, device=dev) * 0.1
    dyo = torch.empty_like(yo)
    dx = torch.empty(B, T, H, W, cin, dtype=torch.bfloat16, device=dev)
    md = B * T * H * W
    part = torch.empty((h._stats_rows(md, plan.d_Npad, plan.d_bn) * 2 * plan.d_Npad,), device=dev)
    fl = 2.0 * plan.M * cout * plan.Ktot
    print(f"{(B, T, H, W, cin)} -> {cout} k{k}: fwd bn {plan.bn}, dgrad bn {plan.d_bn}; {fl / 1e9:.0f} GFLOP",
          flush=True)
    for impl in o.impls:
        wgs = 2 if impl in h._BOX4_IMPLS else 1
        g = h._grid_for(plan.M, plan.Npad, h._box_eff_bn(impl, plan.bn), wgs)
        gd = h._grid_for(md, plan.d_Npad, h._box_eff_bn(impl, plan.d_bn), wgs)
        line = f"impl {impl}:"

        def fwd():
            call("milnce_conv_fwd_pro", ptr(yp), cin, ptr(wp), ptr(y), ptr(stats), None, ptr(ssi), ptr(z),
                 B, T, H, W, cin, cout, *k, *pad, plan.Kpad, plan.Npad, cout, plan.bn, g, impl, stream())

        def dgr():
            call("milnce_conv_dgrad_bnbwd", ptr(dz), ptr(wd), ptr(dx), ptr(part), ptr(yp), ptr(ssi), cin, ptr(yo),
                 ptr(sso), ptr(coef), ptr(dyo), B, T, H, W, cout, cin, *k, *pad, plan.d_Kpad, plan.d_Npad,
                 plan.d_bn, gd, impl, stream())
        for name, fn in (("fwd+pro", fwd), ("dgrad+bnbwd", dgr)):
            try:
                t = timeit(fn, flush)
                line += f"  {name} {t:7.3f} ms {fl / t / 1e9:5.0f} TF/s"
            except h.UnsupportedVariant:
                line += f"  {name} unsupported"
        print(line, flush=True)


if __name__ == "__main__":
    main()

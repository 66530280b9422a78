#!/usr/bin/env python3
"""Time the Inception branch-3 stride-1 max pool at the flagship shapes (bs 256, 16x200x200 input):
forward, plain backward and the fused backward of the model (+ the 1x1 head's dX, + the gate
reduction sum dx * x), for the row sweeps (csrc/pool.hip maxpool_s1_*_rows, impl 2)
and the plane sweeps (impl 1, the default). Pooled values must agree bitwise between
variants (same arg-max); gradients to fp32 rounding (the sweeps sum the scattered gradient in
different orders). "GB/s" counts the bytes each op must move once.

    python tools/pool_bench.py [--only I[,J..]] [--impls 2,1]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mil_nce_howto100m_amd.ops._lib import lib, ptr, stream  # noqa: E402

SHAPES = [(256, 8, 25, 25, 192), (256, 8, 25, 25, 256), (256, 4, 13, 13, 480), (256, 4, 13, 13, 512),
          (256, 4, 13, 13, 528), (256, 2, 7, 7, 832)]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


def main():
    L = lib()
    old = L.milnce_set_pool_s1_impl(1)
    impls = [2, 1]
    if "--impls" in sys.argv:
        impls = [int(v) for v in sys.argv[sys.argv.index("--impls") + 1].split(",")]
    names = {2: "rows", 1: "planes", 0: "slide"}
    print(f"{'shape':28s} {'impl':6s} {'fwd us':>8s} {'bwd us':>8s} {'fused us':>8s} {'GB/s fwd':>9s} "
          f"{'GB/s bwd':>9s} {'GB/s fus':>9s}  check")
    shapes = SHAPES
    if "--only" in sys.argv:
        shapes = [SHAPES[int(i)] for i in sys.argv[sys.argv.index("--only") + 1].split(",")]
    for shp in shapes:
        B, T, H, W, C = shp
        x = torch.randn(*shp, device="cuda").relu().to(torch.bfloat16)  # post-ReLU input: many ties
        dy = torch.randn(*shp, device="cuda").to(torch.bfloat16)
        acc = torch.randn(*shp, device="cuda").to(torch.bfloat16)
        y, dx = torch.empty_like(x), torch.empty_like(x)
        arg = torch.empty(shp, dtype=torch.uint8, device="cuda")
        gs = torch.zeros(B, C, device="cuda")
        geo = [B, T, H, W, C, T, H, W, 3, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0]
        nb = x.numel() * 2
        ref = None
        for impl in impls:
            L.milnce_set_pool_s1_impl(impl)
            fwd = lambda: L.milnce_maxpool_fwd(ptr(x), ptr(y), ptr(arg), *geo, stream())  # noqa: E731
            bwd = lambda: L.milnce_maxpool_bwd(ptr(dy), ptr(arg), ptr(dx), *geo, None, 0, None, None, 2048,  # noqa: E731
                                              stream())
            fus = lambda: L.milnce_maxpool_s1_bwd_fused(ptr(dy), ptr(arg), ptr(acc), ptr(x), ptr(gs), ptr(dx),  # noqa: E731
                                                       B, T, H, W, C, stream())
            tf = timeit(fwd)
            tb = timeit(bwd)
            out = [y.clone(), dx.clone()]
            tu = timeit(fus) if impl >= 1 else float("nan")
            out += [dx.clone(), gs.clone()]
            chk = ""
            if ref is None:
                ref = out
            else:
                assert torch.equal(out[0], ref[0]), (shp, impl, "pooled values differ")
                errs = [rel(a, b) for a, b in zip(out[1:], ref[1:])]
                assert max(errs) < 1e-2, (shp, impl, errs)
                chk = "rel " + " ".join(f"{e:.1e}" for e in errs)
            # fwd: read x, write y + arg; bwd: read dy + arg, write dx; fused: + acc_in, x
            print(f"{str(shp):28s} {names[impl]:6s} {tf * 1e3:8.1f} {tb * 1e3:8.1f} {tu * 1e3:8.1f} "
                  f"{2.5 * nb / tf / 1e6:9.0f} {2.5 * nb / tb / 1e6:9.0f} {4.5 * nb / tu / 1e6:9.0f}  {chk}",
                  flush=True)
    L.milnce_set_pool_s1_impl(old)


if __name__ == "__main__":
    main()

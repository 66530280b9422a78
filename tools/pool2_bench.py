#!/usr/bin/env python3
"""Time the stride-2 TF-SAME pool backwards of the flagship step in isolation (bs 256, 16x200x200):
maxpool_2a (stem output, 1x3x3 / (1,2,2), C 64) and maxpool_3a (conv_2c output, C 192) in the
model's APPLY mode (csrc/pool.hip maxpool_bwd_t MODE 2, QUAD 1: dy of the producer BN from the
pooled gradient, the arg-max codes and the raw conv output), plus the BN-partials pass of the
gated 3a pool (MODE 1), against a plain device copy of the full-resolution tensor (read + write)
as the bandwidth reference. "GB/s" counts the bytes each op must move once.

    python tools/pool2_bench.py [--parts 1024,2048,4096]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import aten  # noqa: E402
from mil_nce_howto100m_amd.ops._lib import lib, ptr, stream  # noqa: E402

SHAPES = [("maxpool_2a", (256, 8, 100, 100, 64)), ("maxpool_3a", (256, 8, 50, 50, 192))]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    L = lib()
    parts = [2048]
    if "--parts" in sys.argv:
        parts = [int(v) for v in sys.argv[sys.argv.index("--parts") + 1].split(",")]
    kernel, strd = (1, 3, 3), (1, 2, 2)
    pads = aten.tf_same_pad(kernel, strd)
    for name, (B, T, H, W, C) in SHAPES:
        To, Ho, Wo = T, (H + 1) // 2, (W + 1) // 2
        geo = [B, T, H, W, C, To, Ho, Wo, *kernel, *strd, pads[0][0], pads[0][1], pads[1][0], pads[1][1],
               pads[2][0], pads[2][1], 1]
        y = torch.randn(B, T, H, W, C, device="cuda").to(torch.bfloat16)
        pooled = torch.empty(B, To, Ho, Wo, C, device="cuda", dtype=torch.bfloat16)
        arg = torch.empty(B, To, Ho, Wo, C, device="cuda", dtype=torch.uint8)
        rc = L.milnce_maxpool_fwd(ptr(y), ptr(pooled), ptr(arg), *geo, stream())
        assert rc == 0, rc
        dout = torch.randn_like(pooled)
        ss = torch.stack([torch.zeros(C), torch.ones(C), torch.rand(C) + 0.5, torch.randn(C) * 0.1]).cuda().reshape(-1)
        coef = (torch.randn(3, C) * 0.1).cuda().reshape(-1)
        g = torch.rand(B, C, device="cuda")
        dmean = torch.randn(B, C, device="cuda")
        out = torch.empty_like(y)
        big = y.numel() * 2
        small = dout.numel() * 2
        copy_us = timeit(lambda: out.copy_(y))
        print(f"{name} {(B, T, H, W, C)}: device copy {copy_us:8.1f} us {2 * big / copy_us / 1e3:7.0f} GB/s",
              flush=True)
        for n in parts:
            ap = lambda: L.milnce_maxpool_bwd_apply(ptr(dout), ptr(arg), ptr(out), *geo, ptr(y), C, ptr(ss),  # noqa
                                                   ptr(coef), None, None, n, stream())
            apg = lambda: L.milnce_maxpool_bwd_apply(ptr(dout), ptr(arg), ptr(out), *geo, ptr(y), C, ptr(ss),  # noqa
                                                    ptr(coef), ptr(g), ptr(dmean), n, stream())
            part = torch.empty(n * 2 * C, device="cuda")
            pg = lambda: L.milnce_maxpool_bwd_gated(ptr(dout), ptr(arg), None, *geo, ptr(y), C, ptr(ss),  # noqa
                                                   ptr(part), n, ptr(g), ptr(dmean), stream())
            t_ap, t_apg = timeit(ap), timeit(apg)
            nb = small + small // 2 + 2 * big  # dout + codes + y + out
            msg = f"  parts {n:5d}: apply {t_ap:8.1f} us {nb / t_ap / 1e3:6.0f} GB/s | gated apply {t_apg:8.1f} us"
            try:
                t_pg = timeit(pg)
                msg += f" | gated partials {t_pg:8.1f} us {(small + small // 2 + big) / t_pg / 1e3:6.0f} GB/s"
            except Exception as e:  # noqa: BLE001
                msg += f" | gated partials: {e}"
            print(msg, flush=True)


if __name__ == "__main__":
    main()

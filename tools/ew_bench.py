#!/usr/bin/env python3
"""Logical streaming bandwidth of the BN / pool kernels at flagship shapes (bs 256, 16x200x200).

Each kernel is timed in isolation on random data; "TB/s" counts the bytes the op must move
(every input read once, every output written once), so it is comparable with the device copy
(``torch.Tensor.copy_``) printed first (MI355X: ~6 TB/s achievable, 8 TB/s peak).

    python tools/ew_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402
from mil_nce_howto100m_amd.ops._lib import call, lib, ptr, stream  # noqa: E402

DEV = "cuda"
BF16 = torch.bfloat16


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def report(name, ms, nbytes):
    print(f"{name:58s} {ms * 1e3:9.1f} us {nbytes / 2**20:9.1f} MiB {nbytes / ms / 1e9:6.2f} TB/s", flush=True)


def bn_ss(C):
    ss = torch.empty(4 * C, device=DEV)
    ss[:C].normal_()
    ss[C:2 * C].uniform_(0.5, 2)
    ss[2 * C:3 * C].uniform_(0.5, 2)
    ss[3 * C:].normal_()
    return ss


def main():
    # baseline: device copy
    for n in (256 * 8 * 2500 * 192, 256 * 4 * 169 * 480):
        x = torch.empty(n, dtype=BF16, device=DEV)
        y = torch.empty_like(x)
        report(f"copy {n * 2 / 2**20:.0f} MiB", timeit(lambda: y.copy_(x)), 4 * n)
        del x, y

    # BN + ReLU apply (train-mode forward of every BN layer that is not fused elsewhere)
    for (B, T, H, W, C) in [(256, 8, 50, 50, 192), (256, 8, 50, 50, 64), (256, 8, 25, 25, 128),
                            (256, 4, 13, 13, 256), (256, 2, 7, 7, 384)]:
        rows = T * H * W
        y = torch.randn(B * rows, C, device=DEV).to(BF16)
        z = torch.empty_like(y)
        ss = bn_ss(C)
        report(f"bn_relu_apply {B}x{T}x{H}x{W}x{C}",
               timeit(lambda: call("milnce_bn_relu_apply", ptr(y), C, ptr(z), C, ptr(ss), C, B, rows, None,
                                   stream())), 4 * y.numel())
        # BN backward apply (partials given): reads dz and y, writes dy
        gamma = torch.rand(C, device=DEV)
        part = torch.randn(2 * C, device=DEV)
        dg, db, coef = torch.empty(C, device=DEV), torch.empty(C, device=DEV), torch.empty(3 * C, device=DEV)
        dy = torch.empty_like(y)
        report(f"bn_bwd (apply) {B}x{T}x{H}x{W}x{C}",
               timeit(lambda: call("milnce_bn_bwd", ptr(z), C, ptr(y), C, ptr(ss), C, B * rows, ptr(gamma),
                                   ptr(part), 1, C, 1, ptr(dg), ptr(db), ptr(coef), ptr(dy), C, 0, 1, stream())),
               6 * y.numel())
        del y, z, dy

    # Inception branch-3 max pool (3,3,3) stride 1, SAME: fwd writes y + uint8 argmax, bwd reads dy + arg
    caps = [int(v) for v in os.environ.get("EW_S1_MAXTHR", "512").split(",")]
    for (B, T, H, W, C), cap in [(s, c) for s in [(256, 8, 25, 25, 192), (256, 8, 25, 25, 256),
                                                   (256, 4, 13, 13, 480), (256, 2, 7, 7, 832)] for c in caps]:
        lib().milnce_set_pool_s1_maxthr(cap)
        x = torch.randn(B, T, H, W, C, device=DEV).to(BF16)
        y = torch.empty_like(x)
        arg = torch.empty(x.shape, dtype=torch.uint8, device=DEV)
        geo = [B, T, H, W, C, T, H, W, 3, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0]
        report(f"maxpool_s1 fwd {B}x{T}x{H}x{W}x{C} cap {cap}",
               timeit(lambda: call("milnce_maxpool_fwd", ptr(x), ptr(y), ptr(arg), *geo, stream())),
               5 * x.numel())
        dx = torch.empty_like(x)
        report(f"maxpool_s1 bwd {B}x{T}x{H}x{W}x{C} cap {cap}",
               timeit(lambda: call("milnce_maxpool_s1_bwd_fused", ptr(y), ptr(arg), None, None, None, ptr(dx),
                                   B, T, H, W, C, stream())), 5 * x.numel())
        del x, y, arg, dx
    lib().milnce_set_pool_s1_maxthr(512)

    # maxpool_3a: (1,3,3) stride (1,2,2) TF-SAME over conv_2c's output
    B, T, H, W, C = 256, 8, 50, 50, 192
    x = torch.randn(B, T, H, W, C, device=DEV).to(BF16)
    To, Ho, Wo = 8, 25, 25
    y = torch.empty(B, To, Ho, Wo, C, dtype=BF16, device=DEV)
    arg = torch.empty(y.shape, dtype=torch.uint8, device=DEV)
    geo = [B, T, H, W, C, To, Ho, Wo, 1, 3, 3, 1, 2, 2, 0, 0, 0, 1, 0, 1, 1]
    report("maxpool (1,3,3)/(1,2,2) fwd 256x8x50x50x192",
           timeit(lambda: call("milnce_maxpool_fwd", ptr(x), ptr(y), ptr(arg), *geo, stream())),
           2 * x.numel() + 3 * y.numel())
    dx = torch.empty_like(x)
    report("maxpool (1,3,3)/(1,2,2) bwd 256x8x50x50x192",
           timeit(lambda: call("milnce_maxpool_bwd", ptr(y), ptr(arg), ptr(dx), *geo, None, 0, None, None, 2048,
                               stream())), 2 * x.numel() + 3 * y.numel())


if __name__ == "__main__":
    lib()
    main()

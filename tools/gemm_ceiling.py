#!/usr/bin/env python3
"""hipBLASLt bf16 GEMM throughput at the conv layers' implicit-GEMM shapes (M = positions,
N = Cout, K = taps * Cin), as a ceiling reference for the conv kernels (no gather, no epilogue).

    python tools/gemm_ceiling.py
"""
import torch


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


SHAPES = [  # (M, N, K, what)
    (256 * 8 * 50 * 50, 192, 576, "conv_2c spatial fwd (64->192, 1x3x3)"),
    (256 * 8 * 50 * 50, 192, 576, "conv_2c temporal fwd (192->192, 3x1x1)"),
    (256 * 8 * 50 * 50, 64, 1728, "conv_2c spatial dgrad (192->64)"),
    (256 * 8 * 25 * 25, 192, 1152, "3c b1b spatial fwd (128->192)"),
    (256 * 8 * 25 * 25, 288, 256, "3b head 1x1 (256->288)"),
    (8192, 8192, 8192, "square 8192"),
]

for M, N, K, what in SHAPES:
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    ms = timeit(lambda: torch.mm(a, w.t()))
    print(f"{what:42s} M {M:8d} N {N:5d} K {K:5d}: {ms:7.3f} ms {2.0 * M * N * K / ms / 1e9:7.0f} TF/s", flush=True)
    del a, w

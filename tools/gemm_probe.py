#!/usr/bin/env python3
"""Library GEMM (torch.mm -> hipBLASLt) time for the Inception head 1x1 convs at bs 256
(M x K @ K x N, bf16), next to the bytes / FLOP floors: is a library GEMM + a statistics pass
cheaper than the fused conv kernels for these shapes?"""
import torch

HEADS = {"3b": (1280000, 192, 176), "3c": (1280000, 256, 288), "4b": (173056, 480, 304),
         "4c": (173056, 512, 296), "4d": (173056, 512, 280), "4e": (173056, 512, 288),
         "4f": (173056, 528, 448), "5b": (25088, 832, 448), "5c": (25088, 832, 624)}


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for name, (M, K, N) in HEADS.items():
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    t = timeit(lambda: torch.mm(x, w.t(), out=y))
    ts = timeit(lambda: y.float().sum(0))
    floor = (M * K + M * N) * 2 / 5e12 * 1e6
    print(f"{name}: M {M} K {K} N {N}: mm {t:7.1f} us  (sum pass {ts:6.1f} us)  5TB/s floor {floor:6.1f} us  "
          f"{2 * M * K * N / t / 1e6:6.0f} TF/s", flush=True)

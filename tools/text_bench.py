#!/usr/bin/env python3
"""Fused text-tower forward kernel (gather + fc1 + bias + ReLU + max over words) vs the unfused
sequence it replaces (index_select + hipBLASLt addmm + ReLU-max kernel) at the flagship shape
(256 clips x 4 candidate captions, 20 words, 300 -> 2048).

    python tools/text_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402
from mil_nce_howto100m_amd.ops._lib import call, ptr, stream  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    N, Wd, V, D, F = 1024, 20, 66250, 300, 2048
    tok = torch.randint(0, V, (N, Wd), device="cuda")
    table = torch.randn(V, D, device="cuda")
    tp = h.text_table_padded(table)
    tb = table.to(torch.bfloat16)
    w1 = torch.randn(F, D, device="cuda") * 0.05
    b1 = torch.randn(F, device="cuda")
    w1p = torch.zeros((F, tp.shape[1]), dtype=torch.bfloat16, device="cuda")
    w1p[:, :D] = w1
    hm = torch.empty((N, F), device="cuda")
    arg = torch.empty((N, F), dtype=torch.uint8, device="cuda")

    def fused():
        call("milnce_text_fc1_max", ptr(tok), N, Wd, ptr(tp), ptr(w1p), ptr(b1), F, tp.shape[1], ptr(hm), ptr(arg),
             stream())

    def unfused():
        e = tb.index_select(0, tok.reshape(-1))
        hh = torch.addmm(b1.to(torch.bfloat16), e, w1.to(torch.bfloat16).t())
        call("milnce_text_relu_max", ptr(hh), N, Wd, F, ptr(hm), ptr(arg), stream())

    fl = 2.0 * N * Wd * F * D
    tf, tu = timeit(fused), timeit(unfused)
    print(f"fused   {tf:7.1f} us ({fl / tf / 1e6:6.1f} TF/s)")
    print(f"unfused {tu:7.1f} us (index_select + addmm + relu-max)")


if __name__ == "__main__":
    main()

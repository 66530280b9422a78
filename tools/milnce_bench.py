#!/usr/bin/env python3
"""Fused vs materialised MIL-NCE, forward + backward, at the BASELINE global batches.

    python tools/milnce_bench.py [--B 2048 8192] [--K 4] [--reps 5]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, nargs="+", default=[2048, 8192])
    ap.add_argument("--K", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    o = ap.parse_args()
    from mil_nce_howto100m_amd.ops import hip_ops as h
    for B in o.B:
        v = (torch.randn(B, 512, device="cuda") * 0.05).requires_grad_(True)
        t = (torch.randn(B * o.K, 512, device="cuda") * 0.05).requires_grad_(True)
        res = {}
        for fused in (True, False):
            ts = []
            for _ in range(o.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                h.milnce_loss(v, t, fused=fused).backward()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
            res[fused] = min(ts[1:])
        print(f"B {B} K {o.K}: fused {res[True]:.3f} ms, materialised {res[False]:.3f} ms", flush=True)


if __name__ == "__main__":
    main()

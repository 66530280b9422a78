#!/usr/bin/env python3
"""Run the paired-width stem forward / wgrad kernels at the flagship shape (for rocprofv3 passes).

    python tools/stem_probe.py [--batch 256] [--frames 16] [--size 200]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--size", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    o = ap.parse_args()
    S, W2 = o.size, o.size // 2
    x2 = torch.randn(o.batch, o.frames, S, W2, 8, device="cuda").to(torch.bfloat16)
    w2 = torch.randn(64, 8, 3, 7, 4, device="cuda") * 0.05
    plan = h.conv_plan(x2.shape, w2.shape, (2, 2, 1), (1, 3, 2), W2)
    wp = h._pack(w2, plan, 0)
    stats = torch.empty((h._stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad,), device="cuda")
    y = h.conv_forward_raw(x2, wp, plan, stats)
    dy = torch.randn_like(y)
    from mil_nce_howto100m_amd.ops._lib import lib, ptr, stream
    st2 = torch.empty((256 * 128,), device="cuda")
    for _ in range(o.reps):
        h.conv_forward_raw(x2, wp, plan, stats)  # generic implicit GEMM
        lib().milnce_stem_fwd(ptr(x2), 0, ptr(wp), plan.Kpad, ptr(y), ptr(st2), st2.numel(), None, plan.B, plan.T, plan.H,
                              plan.W, stream())  # halo kernel
        h.conv_wgrad(dy, x2, plan)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Time the uint8 stem forward (csrc/conv.hip stem_fwd_kernel) at the flagship shape, for A/B
libraries (MILNCE_LIB_PATH, e.g. the STEM_ABLATE builds: python csrc/build.py --define STEM_ABLATE=1).

    MILNCE_LIB_PATH=... python tools/stem_fwd_ab.py [--batch 256]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402
from mil_nce_howto100m_amd.ops._lib import lib, ptr, stream, LIB_PATH  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    o = ap.parse_args()
    B, T, S, W2 = o.batch, 16, 200, 100
    x = torch.randint(0, 255, (B, T, S, W2, 8), device="cuda", dtype=torch.uint8)
    w2 = torch.randn(64, 8, 3, 7, 4, device="cuda") * 0.05
    plan = h.conv_plan((B, T, S, W2, 8), w2.shape, (2, 2, 1), (1, 3, 2), W2)
    wp = h._pack(w2, plan, 0)
    y = torch.empty((plan.M, 64), device="cuda", dtype=torch.bfloat16)
    st = torch.empty((256 * 128,), device="cuda")
    f = lambda: lib().milnce_stem_fwd(ptr(x), 1, ptr(wp), plan.Kpad, ptr(y), ptr(st), st.numel(), None,  # noqa: E731
                                      B, T, S, W2, stream())
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(o.reps):
        f()
    b.record()
    b.synchronize()
    print(f"{os.path.basename(LIB_PATH)}: stem fwd {a.elapsed_time(b) / o.reps:.3f} ms", flush=True)


if __name__ == "__main__":
    main()

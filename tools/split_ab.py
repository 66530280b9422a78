#!/usr/bin/env python3
"""Time the halo and temporal box wgrads at the flagship shapes for every occupancy target, to
compare the split-count rule (csrc/common.h fill_splits; run once with MILNCE_SPLIT_CEIL=1 for the
rounded-up count). Prints workgroups launched and us per call.

    python tools/split_ab.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402

SHAPES = [(256, 8, 50, 50, 64, 192, (1, 3, 3)), (256, 8, 50, 50, 192, 192, (3, 1, 1)),
          (256, 8, 25, 25, 128, 192, (1, 3, 3)), (256, 8, 25, 25, 96, 208, (1, 3, 3)),
          (256, 8, 25, 25, 128, 192, (3, 1, 1)), (256, 4, 13, 13, 112, 224, (1, 3, 3))]


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    mode = "ceil" if os.environ.get("MILNCE_SPLIT_CEIL") == "1" else "floor"
    for B, T, H, W, Cin, Cout, k in SHAPES:
        pad = tuple(kk // 2 for kk in k)
        x = torch.randn(B, T, H, W, Cin, device="cuda").to(torch.bfloat16)
        dy = torch.randn(B, T, H, W, Cout, device="cuda").to(torch.bfloat16)
        plan = h.conv_plan(x.shape, (Cout, Cin) + k, (1, 1, 1), pad)
        out = torch.zeros((Cout, Cin) + k, device="cuda")
        res = []
        for occ in (1, 2, 4, 8):
            t = timeit(lambda: h._halo_wgrad(dy, x, plan, 64, out, 0, occ))
            res.append(f"halo o{occ} {t:7.1f}")
        if k == (3, 1, 1):
            for reg in (1, 2):
                for bn in h._tw_tiles(Cout):
                    for occ in (1, 2):
                        t = timeit(lambda: h._twgrad(dy, x, plan, bn, out, 0, occ, reg))
                        res.append(f"tw{reg}/{bn}/o{occ} {t:7.1f}")
        print(f"[{mode}] {(T, H, W, Cin)}->{Cout} k{k}: " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()

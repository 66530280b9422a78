#!/usr/bin/env python3
"""Time the Inception branch-3 stride-1 max pool (forward and backward) at the flagship shapes
(bs 256, 16x200x200 input) for both implementations: LDS plane sweep vs global sliding window.

    python tools/pool_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402
from mil_nce_howto100m_amd.ops._lib import lib  # noqa: E402

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


def main():
    L = lib()
    print(f"{'shape':32s} {'impl':6s} {'fwd us':>8s} {'bwd us':>8s} {'GB/s fwd':>9s} {'GB/s bwd':>9s}")
    for shp in SHAPES:
        x = torch.randn(*shp, device="cuda").to(torch.bfloat16)
        dy = torch.randn(*shp, device="cuda").to(torch.bfloat16)
        nb = x.numel() * 2
        for impl, name in ((1, "lds"), (0, "slide")):
            L.milnce_set_pool_s1_impl(impl)
            xr = x.clone().requires_grad_(True)
            f = lambda: h.maxpool3d(xr, (3, 3, 3), (1, 1, 1), False)  # noqa: E731
            tf = timeit(f)
            y = f()
            tb = timeit(lambda: torch.autograd.grad(y, xr, dy, retain_graph=True))
            # fwd: read x, write y + arg; bwd: read dy + arg, write dx
            print(f"{str(shp):32s} {name:6s} {tf * 1e3:8.1f} {tb * 1e3:8.1f} {2.5 * nb / tf / 1e6:9.0f} "
                  f"{2.5 * nb / tb / 1e6:9.0f}")
    L.milnce_set_pool_s1_impl(1)


if __name__ == "__main__":
    main()

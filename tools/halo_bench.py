#!/usr/bin/env python3
"""Time the box-tiled halo kernels against the tuned im2col kernels on the flagship conv shapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402

SHAPES = [(256, 8, 50, 50, 64, 192, (1, 3, 3)), (256, 8, 50, 50, 192, 192, (3, 1, 1)),
          (256, 8, 25, 25, 128, 192, (1, 3, 3)), (256, 8, 25, 25, 96, 128, (1, 3, 3)),
          (256, 8, 25, 25, 192, 192, (3, 1, 1)), (256, 4, 13, 13, 160, 320, (1, 3, 3)),
          (256, 4, 13, 13, 320, 320, (3, 1, 1)), (256, 2, 7, 7, 192, 384, (1, 3, 3)),
          (256, 8, 25, 25, 128, 128, (3, 1, 1)), (256, 4, 13, 13, 288, 288, (3, 1, 1)),
          (256, 2, 7, 7, 384, 384, (3, 1, 1))]


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


for B, T, H, W, Cin, Cout, k in SHAPES:
    pad = tuple(kk // 2 for kk in k)
    x = torch.randn(B, T, H, W, Cin, device="cuda").to(torch.bfloat16)
    dy = torch.randn(B, T, H, W, Cout, device="cuda").to(torch.bfloat16)
    plan = h.conv_plan(x.shape, (Cout, Cin) + k, (1, 1, 1), pad)
    fl = 2.0 * plan.M * Cout * Cin * k[0] * k[1] * k[2]
    out = torch.zeros((Cout, Cin) + k, device="cuda")
    h._HALO_WGRAD = False
    plan.w_impl = 0
    t_old = timeit(lambda: h.conv_wgrad(dy, x, plan))
    res = [f"im2col {t_old:.3f} ms {fl / t_old / 1e9:.0f} TF/s"]
    for cc in ((64,) if k[0] == 1 else (128, 64)):
        t = timeit(lambda: h._halo_wgrad(dy, x, plan, cc, out, 0))
        res.append(f"halo cc{cc} {t:.3f} ms {fl / t / 1e9:.0f} TF/s")
    if k == (3, 1, 1):  # temporal box wgrad (csrc/conv_twgrad.hip), output tile x workgroups per CU
        for reg in (0, 1):
            for bn in h._tw_tiles(Cout):
                for occ in (1, 2):
                    t = timeit(lambda: h._twgrad(dy, x, plan, bn, out, 0, occ, reg))
                    res.append(f"tw{'r' if reg else ''}{bn}/o{occ} {t:.3f} ms {fl / t / 1e9:.0f} TF/s")
    print(f"{(B, T, H, W, Cin)}->{Cout} k{k}: " + " | ".join(res), flush=True)

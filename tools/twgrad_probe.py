#!/usr/bin/env python3
"""Launch the temporal box wgrad (csrc/conv_twgrad.hip) and the im2col wgrad on one (3,1,1) shape a
few times (for rocprofv3 counter passes: tools/gpu/tw_pmc.sh).

    python tools/twgrad_probe.py [--cin 192 --cout 192 --t 8 --hw 50 --bn 192 --occ 2 --reps 3]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=192)
    ap.add_argument("--cout", type=int, default=192)
    ap.add_argument("--t", type=int, default=8)
    ap.add_argument("--hw", type=int, default=50)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--bn", type=int, default=192)
    ap.add_argument("--occ", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--time", type=str, default="",
                    help="comma list of reg modes (0 DMA, 1 register ring, 2 pipelined) to time instead")
    o = ap.parse_args()
    x = torch.randn(o.batch, o.t, o.hw, o.hw, o.cin, device="cuda").to(torch.bfloat16)
    dy = torch.randn(o.batch, o.t, o.hw, o.hw, o.cout, device="cuda").to(torch.bfloat16)
    plan = h.conv_plan(x.shape, (o.cout, o.cin, 3, 1, 1), (1, 1, 1), (1, 0, 0))
    out = torch.zeros((o.cout, o.cin, 3, 1, 1), device="cuda")
    if o.time:
        for reg in [int(v) for v in o.time.split(",")]:
            for occ in (1, 2):
                fn = lambda: h._twgrad(dy, x, plan, o.bn, out, 0, occ, reg)  # noqa: E731
                fn()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(10):
                    fn()
                b.record()
                b.synchronize()
                us = a.elapsed_time(b) / 10 * 1e3
                tf = 2.0 * o.batch * o.t * o.hw * o.hw * o.cout * o.cin * 3 / us / 1e6
                print(f"bn {o.bn} reg {reg} occ {occ}: {us:8.1f} us {tf:7.1f} TFLOP/s", flush=True)
        return
    h._HALO_WGRAD = False
    h._TWGRAD = False
    plan.w_impl = 0
    for _ in range(o.reps):
        h.conv_wgrad(dy, x, plan)  # im2col (tuned once)
        h._twgrad(dy, x, plan, o.bn, out, 0, o.occ)
    torch.cuda.synchronize()
    print("done", plan.w_impl, plan.w_tn, plan.w_tk)


if __name__ == "__main__":
    main()

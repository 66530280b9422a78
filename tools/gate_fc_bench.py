"""Isolated timing of the SelfGating fc kernels (csrc/gate.hip gate_fc_kernel / gate_fc_bwd_kernel)
on the S3D-G gating shapes at B clips: python tools/gate_fc_bench.py [--B 256]
(MILNCE_LIB_PATH selects the library, for A/Bs)."""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mil_nce_howto100m_amd.ops._lib import call, ptr, stream  # noqa: E402

SHAPES = {"conv_2c": (192,), "mixed_3b": (64, 128, 32, 32), "mixed_3c": (128, 192, 96, 64),
          "mixed_4b": (192, 208, 48, 64), "mixed_4f": (256, 320, 128, 128), "mixed_5c": (384, 384, 128, 128)}


def arr(t, vals):
    return (t * len(vals))(*vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    B, dev = a.B, "cuda"
    torch.manual_seed(0)
    tot_f = tot_b = 0.0
    for name, widths in SHAPES.items():
        n, Ct = len(widths), sum(widths)
        ws = [torch.randn(c, c, device=dev) * 0.05 for c in widths]
        bs = [torch.randn(c, device=dev) for c in widths]
        dws = [torch.zeros(c, c, device=dev) for c in widths]
        dbs = [torch.zeros(c, device=dev) for c in widths]
        gsum = torch.rand(B, Ct, device=dev) * 100
        mean = torch.empty(B, Ct, device=dev)
        g = torch.empty(B, Ct, device=dev)
        src = torch.randn(B, Ct, device=dev)
        dmean = torch.empty(B, Ct, device=dev)
        wa = arr(ctypes.c_void_p, [w.data_ptr() for w in ws])
        ba = arr(ctypes.c_void_p, [b.data_ptr() for b in bs])
        dwa = arr(ctypes.c_void_p, [w.data_ptr() for w in dws])
        dba = arr(ctypes.c_void_p, [b.data_ptr() for b in dbs])
        wid = arr(ctypes.c_int, widths)

        def fwd():
            call("milnce_gate_fwd", n, wid, None, wa, ba, ptr(gsum), B, 100, ptr(mean), ptr(g), None, None, None,
                 None, None, 0, stream())

        def bwd():
            call("milnce_gate_fc_bwd", n, wid, ptr(src), ptr(g), ptr(mean), wa, dwa, dba, 0, B, ptr(dmean), stream())

        res = []
        for fn in (fwd, bwd):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                fn()
            e1.record()
            e1.synchronize()
            res.append(e0.elapsed_time(e1) / a.reps * 1e3)
        # check against torch
        want_g = torch.cat([torch.sigmoid(mean[:, o:o + c] @ w.t() + b) for w, b, c, o in
                            zip(ws, bs, widths, [sum(widths[:i]) for i in range(n)])], 1)
        errg = ((g - want_g).abs().max()).item()
        d = src * (1 - g)
        want_dm = torch.cat([d[:, o:o + c] @ w for w, c, o in zip(ws, widths, [sum(widths[:i]) for i in range(n)])], 1)
        errm = ((dmean - want_dm).abs().max() / want_dm.abs().max()).item()
        o0 = 0
        errw = 0.0
        for w, dw, db, c in zip(ws, dws, dbs, widths):
            ref = d[:, o0:o0 + c].t() @ mean[:, o0:o0 + c]
            errw = max(errw, ((dw - ref).abs().max() / ref.abs().max()).item())
            errw = max(errw, ((db - d[:, o0:o0 + c].sum(0)).abs().max() / d[:, o0:o0 + c].sum(0).abs().max()).item())
            o0 += c
        tot_f += res[0]
        tot_b += res[1]
        print(f"{name:9s} fc fwd {res[0]:7.1f} us  fc bwd {res[1]:7.1f} us   err g {errg:.1e} dmean {errm:.1e} dW/db {errw:.1e}")
    print(f"total     fc fwd {tot_f:7.1f} us  fc bwd {tot_b:7.1f} us")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where a box-tiled conv tile's time goes: per-phase s_memtime stamps of csrc/conv_box.hip built
with -DBOX_TRACE=1 (``python csrc/build.py --trace`` -> libmilnce_hip_trace.so).

    MILNCE_LIB_PATH=.../libmilnce_hip_trace.so python tools/box_trace.py [--cin 64 --cout 192 --k 1 3 3
        --hw 50 --impl 15 --dir fwd|dgrad --producer 0|1]

Every wave of the first 64 workgroups records, per tap: W (its weight-stage wait returned), B (ring
barrier passed), M (the tap's fragment reads + MFMAs issued); per block: X (block-end barrier), S
(next block's box written); per epilogue half: H1 (rows staged + barrier), H2 (stores issued), H3
(barrier); N (next tile's box written). Printed: mean cycles per phase for tiles 1.. (tile 0 holds the
prologue), over waves, and the max-over-waves view that the barriers impose.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import _lib  # noqa: E402
from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402


def decode(ev, n, ncb, taps):
    """events of one wave -> list of per-tile dicts of phase durations (cycles)."""
    ev = ev[:min(n, 128)]
    tiles = []
    i = 1  # event 0: setup done
    prev = ev[0] if len(ev) else 0
    per_tile = ncb * (3 * taps + 1) + (ncb - 1) + 7
    while i + per_tile <= len(ev):
        d = {"wait": 0, "barrier": 0, "mfma": 0, "blockend": 0, "boxstore": 0}
        for cb in range(ncb):
            for t in range(taps):
                w, b, m = ev[i], ev[i + 1], ev[i + 2]
                d["wait"] += w - prev
                d["barrier"] += b - w
                d["mfma"] += m - b
                prev = m
                i += 3
            d["blockend"] += ev[i] - prev
            prev = ev[i]
            i += 1
            if cb < ncb - 1:
                d["boxstore"] += ev[i] - prev
                prev = ev[i]
                i += 1
        for half in range(2):
            h1, h2, h3 = ev[i], ev[i + 1], ev[i + 2]
            d[f"stage{half}"] = h1 - prev
            d[f"stores{half}"] = h2 - h1
            d[f"bar{half}"] = h3 - h2
            prev = h3
            i += 3
        d["nextbox"] = ev[i] - prev
        prev = ev[i]
        i += 1
        d["total"] = sum(v for k, v in d.items())
        tiles.append(d)
    return tiles


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=64)
    ap.add_argument("--cout", type=int, default=192)
    ap.add_argument("--k", type=int, nargs=3, default=[1, 3, 3])
    ap.add_argument("--t", type=int, default=8)
    ap.add_argument("--hw", type=int, default=50)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--impl", type=int, default=15)
    ap.add_argument("--dir", default="fwd")
    ap.add_argument("--producer", type=int, default=1)
    o = ap.parse_args()
    lib = _lib.lib()
    buf = torch.zeros(64 * 8 * 130, dtype=torch.int32, device="cuda")
    if lib.milnce_box_set_trace(buf.data_ptr()) != 0:
        sys.exit("the loaded library is not a BOX_TRACE build (python csrc/build.py --trace; MILNCE_LIB_PATH)")
    k = tuple(o.k)
    pad = tuple(kk // 2 for kk in k)
    x = torch.randn(o.batch, o.t, o.hw, o.hw, o.cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(o.cout, o.cin, *k, device="cuda") * 0.05
    plan = h.conv_plan(x.shape, w.shape, (1, 1, 1), pad)
    wp, wd = h._pack(w, plan, 0), h._pack(w, plan, 1)
    stats = torch.empty((h._stats_rows(plan.M, plan.Npad, plan.bn) * 2 * plan.Npad,), device="cuda")
    dy = torch.randn(plan.B, plan.To, plan.Ho, plan.Wo, o.cout, device="cuda").to(torch.bfloat16)
    ss = torch.cat([torch.zeros(o.cin, device="cuda"), torch.ones(o.cin, device="cuda"),
                    torch.ones(o.cin, device="cuda"), torch.zeros(o.cin, device="cuda")])
    prod = (x, ss, o.cin) if o.producer else None
    plan.pin_f = plan.pin_d = o.impl
    plan.grid_m = h._grid_for(plan.M, plan.Npad, plan.bn, 1)
    plan.d_grid_m = h._grid_for(plan.B * plan.T * plan.H * plan.W, plan.d_Npad, plan.d_bn, 1)
    if o.dir == "fwd":
        run = lambda: h.conv_forward_raw(x, wp, plan, stats)  # noqa: E731
        cin_eff, bn = o.cin, plan.bn
    else:
        run = lambda: h.conv_dgrad(dy, wd, plan, prod)  # noqa: E731
        cin_eff, bn = o.cout, plan.d_bn
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    run()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b)
    tr = buf.view(64, 8, 130).cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    taps = k[0] * k[1] * k[2]
    ncb = int(tr[0, 0, 129])
    allt = []
    for g in range(64):
        for wv in range(8):
            tiles = decode(tr[g, wv, :128], int(tr[g, wv, 128]), ncb, taps)
            allt += tiles[1:]
    print(f"{o.dir} {tuple(x.shape)} -> {o.cout} k{k} impl {o.impl} bn {bn}: {ms:.3f} ms, ncb {ncb}, "
          f"{len(allt)} wave-tiles decoded")
    if not allt:
        return
    keys = list(allt[0].keys())
    tot = np.mean([t["total"] for t in allt])
    for kk in keys:
        v = np.array([t[kk] for t in allt], dtype=np.float64)
        print(f"  {kk:10s} mean {v.mean():9.0f} cyc  p90 {np.percentile(v, 90):9.0f}  {100 * v.mean() / tot:5.1f} %")


if __name__ == "__main__":
    main()

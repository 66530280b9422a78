#!/usr/bin/env python3
"""Per-queue kernel-class totals of the last step(s) of a rocprofv3 kernel trace (bench.py run).

    python tools/step_classes.py run_kernel_trace.csv [--steps 2]

The step boundary is the synthetic-batch kernel (synth_video_kernel, one per step); classes:
conv fwd/dgrad, wgrad, pool, BN, gate, other. Main queue = the one with the most dispatches.
"""
import csv
import sys
from collections import defaultdict


def klass(name):
    n = name.split("(")[0]
    if "wgrad" in n or "twgrad" in n or "reduce_batch" in n:
        return "wgrad"
    if n.startswith(("void conv_", "conv_", "void stem_fwd", "stem_fwd")):
        return "conv fwd/dgrad"
    if "pool" in n:
        return "pool"
    if n.startswith(("bn_", "void bn_")):
        return "bn"
    if n.startswith(("gate_", "void gate_")):
        return "gate"
    return "other"


def main(path, steps=2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("synth_video_kernel")]
    if len(starts) < steps + 1:
        sel = rows[starts[-steps]:] if len(starts) >= steps else rows
    else:
        sel = rows[starts[-steps - 1]:starts[-1]]
    nsteps = steps
    qcount = defaultdict(int)
    for r in sel:
        qcount[r["Queue_Id"]] += 1
    main_q = max(qcount, key=qcount.get)
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for r in sel:
        q = "main" if r["Queue_Id"] == main_q else "side"
        k = klass(r["Kernel_Name"])
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[(q, k)] += us
        cnt[(q, k)] += 1
    wall = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e6 / nsteps
    print(f"{nsteps} step(s), wall {wall:.2f} ms/step")
    for q in ("main", "side"):
        s = sum(v for (qq, _), v in tot.items() if qq == q) / 1e3 / nsteps
        print(f"{q}: {s:.2f} ms/step")
        for (qq, k), v in sorted(tot.items(), key=lambda kv: -kv[1]):
            if qq == q:
                print(f"   {k:16s} {v / 1e3 / nsteps:7.2f} ms  {cnt[(qq, k)] / nsteps:6.1f} calls")


if __name__ == "__main__":
    a = sys.argv[1:]
    st = 2
    if "--steps" in a:
        st = int(a[a.index("--steps") + 1])
    main(a[0], st)

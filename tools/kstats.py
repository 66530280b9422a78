#!/usr/bin/env python3
"""Summarise rocprofv3 output: ms per step per kernel (top N).

    kstats.py run_kernel_stats.csv STEPS [TOP]            # whole-run stats / STEPS
    kstats.py run_kernel_trace.csv --skip S [--top N]     # trace: drop the first S steps (warmup,
                                                          # autotuning); steps delimited by the
                                                          # once-per-step synth_video kernel
"""
import argparse
import csv
from collections import defaultdict


def from_trace(path, skip, top, marker="synth_video"):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(marker)]
    if len(starts) <= skip:
        raise SystemExit(f"only {len(starts)} steps in trace")
    sel = rows[starts[skip]:]
    steps = len(starts) - skip
    agg, cnt = defaultdict(float), defaultdict(int)
    for r in sel:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[r["Kernel_Name"]] += d
        cnt[r["Kernel_Name"]] += 1
    wall = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e6 / steps
    tot = sum(agg.values())
    print(f"{steps} steps: GPU kernel time {tot / 1e6 / steps:.2f} ms/step, first-to-last wall {wall:.2f} ms/step")
    print(f"{'ms/step':>8} {'calls/step':>10} {'avg_us':>8}  kernel")
    for k, t in sorted(agg.items(), key=lambda kv: -kv[1])[:top]:
        print(f"{t / 1e6 / steps:8.2f} {cnt[k] / steps:10.1f} {t / cnt[k] / 1e3:8.1f}  {k[:100]}")
    return agg, cnt, steps


def from_stats(path, steps, top):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total GPU kernel time per step: {tot / 1e6 / steps:.2f} ms over {len(rows)} kernels")
    print(f"{'ms/step':>8} {'calls/step':>10} {'avg_us':>8}  kernel")
    for r in rows[:top]:
        t, c = float(r["TotalDurationNs"]), float(r["Calls"])
        print(f"{t / 1e6 / steps:8.2f} {c / steps:10.1f} {t / c / 1e3:8.1f}  {r['Name'][:100]}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("steps", nargs="?", type=float, default=1.0)
    ap.add_argument("top_pos", nargs="?", type=int, default=None)
    ap.add_argument("--skip", type=int, default=None)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    top = a.top_pos or a.top
    if a.skip is not None:
        from_trace(a.path, a.skip, top)
    else:
        from_stats(a.path, a.steps, top)

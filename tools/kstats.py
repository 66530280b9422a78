#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats CSV: ms per step per kernel (top N)."""
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total GPU kernel time per step: {tot / 1e6 / steps:.2f} ms over {len(rows)} kernels")
print(f"{'ms/step':>8} {'calls/step':>10} {'avg_us':>8}  kernel")
for r in rows[:top]:
    t = float(r["TotalDurationNs"])
    c = float(r["Calls"])
    print(f"{t / 1e6 / steps:8.2f} {c / steps:10.1f} {t / c / 1e3:8.1f}  {r['Name'][:100]}")

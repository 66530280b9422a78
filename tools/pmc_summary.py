#!/usr/bin/env python3
"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv: kstats-style summary.

    pmc_summary.py run_counter_collection.csv [name-substring]
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
for r in rows:
    name = r["Kernel_Name"].split("(")[0][:60]
    if sub not in r["Kernel_Name"]:
        continue
    agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[name][r["Counter_Name"]] += 1
for name, d in agg.items():
    print(name)
    for k, v in sorted(d.items()):
        print(f"   {k:32s} {v / cnt[name][k]:16.1f}  (avg over {cnt[name][k]} dispatches)")

#!/usr/bin/env python3
"""Per-kernel-name counter summary of a directory of rocprofv3 CSV runs (tools/gpu/conv_pmc.sh).

Averages every counter over the dispatches of each kernel name and prints derived ratios:
wave-cycle shares (wait / issue-stall / active), MFMA busy share of GRBM cycles, LDS conflicts.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0][:70]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0][:70]
            durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, c in vals.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        us = sorted(durs.get(k, [0.0]))[len(durs.get(k, [0.0])) // 2]
        print(f"== {k}  median {us:.1f} us")
        for n in sorted(m):
            print(f"   {n:32s} {m[n]:16.1f}")
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            print(f"   wait {m.get('SQ_WAIT_ANY', 0) / wc:.2f}  stall {m.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}  "
                  f"active {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}  lds-stall {m.get('SQ_WAIT_INST_LDS', 0) / wc:.2f}")
        g = m.get("GRBM_GUI_ACTIVE", 0.0)
        if g and us:
            print(f"   clock {g / 8 / us / 1e3:.2f} GHz")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and g:
            print(f"   mfma busy share {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 256 * 4):.3f} (per SIMD)")
        if m.get("SQ_LDS_IDX_ACTIVE") and g:
            print(f"   lds active share {m['SQ_LDS_IDX_ACTIVE'] / (g / 8 * 256):.3f} (per CU, raw units)")
        if m.get("SQ_INSTS_MFMA"):
            print(f"   valu/mfma {m.get('SQ_INSTS_VALU', 0) / m['SQ_INSTS_MFMA']:.2f}  "
                  f"lds/mfma {m.get('SQ_INSTS_LDS', 0) / m['SQ_INSTS_MFMA']:.2f}  "
                  f"vmem/mfma {m.get('SQ_INSTS_VMEM', 0) / m['SQ_INSTS_MFMA']:.2f}")
        if m.get("SQ_LDS_IDX_ACTIVE"):
            print(f"   lds conflict ratio {m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_LDS_IDX_ACTIVE']:.3f}")


if __name__ == "__main__":
    main(sys.argv[1])

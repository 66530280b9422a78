#!/usr/bin/env python3
"""Estimated occupancy (waves per SIMD) of every kernel in a rocprofv3 kernel trace, from its
VGPR/AGPR allocation, LDS per workgroup and workgroup size (MI355X: 512 regs/lane/SIMD in 8-reg
granules, 160 KiB LDS, 32 waves/CU), weighted by time: which kernels run at 1 wave/SIMD.

    occupancy.py run_kernel_trace.csv [--top N]
"""
import argparse
import csv
from collections import defaultdict


def waves_per_simd(vgpr, agpr, lds, wg):
    regs = vgpr + agpr
    alloc = max(8, (regs + 7) // 8 * 8)
    by_regs = min(8, 512 // alloc)
    waves_per_wg = max(1, (wg + 63) // 64)
    by_lds = (160 * 1024) // lds if lds > 0 else 99
    wgs = min(by_lds, (by_regs * 4) // waves_per_wg, 32 // waves_per_wg)
    return min(by_regs, wgs * waves_per_wg / 4.0), by_regs, by_lds


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    t = defaultdict(float)
    info = {}
    for r in csv.DictReader(open(a.trace)):
        k = r["Kernel_Name"].split("(")[0][:70]
        t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        info[k] = (int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"]), int(r["LDS_Block_Size"]),
                   int(r["Workgroup_Size_X"]), int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
    print(f"{'ms':>8} {'waves/SIMD':>10} {'regs':>6} {'LDS KiB':>8} {'wg':>5} {'grid':>7}  kernel")
    for k, ms in sorted(t.items(), key=lambda kv: -kv[1])[:a.top]:
        v, ag, lds, wg, grid = info[k]
        occ, _, _ = waves_per_simd(v, ag, lds, wg)
        print(f"{ms:8.2f} {occ:10.2f} {v + ag:6d} {lds / 1024:8.1f} {wg:5d} {grid:7d}  {k}")


if __name__ == "__main__":
    main()

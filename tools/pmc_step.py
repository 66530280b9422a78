#!/usr/bin/env python3
"""Per-kernel hardware counters for ONE flagship training step (the last step of the run).

    pmc_step.py --trace run_kernel_trace.csv --pmc a.csv b.csv ... [--top N]

Every input is a rocprofv3 CSV of the same program (`bench.py --steps 1 --warmup 1`). Steps are
delimited by the once-per-step ``synth_video`` kernel, so autotuning trials of the warmup step are
dropped. Per kernel name it reports: calls, ms/step (trace), MFMA utilisation (``MfmaUtil``), LDS
bank-conflict cycles per LDS-active cycle, HBM bytes (FETCH_SIZE + WRITE_SIZE, KiB) and the
achieved HBM bandwidth that implies against the traced duration.
"""
import argparse
import csv
from collections import defaultdict

MARKER = "synth_video"


def last_step_rows(rows, key):
    rows.sort(key=key)
    starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(MARKER)]
    if not starts:
        raise SystemExit("no step marker kernel found")
    return rows[starts[-1]:]


def short(name, n=58):
    return name.split("(")[0][:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--pmc", nargs="+", required=True)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()

    tr = last_step_rows(list(csv.DictReader(open(a.trace))), lambda r: int(r["Start_Timestamp"]))
    dur, calls = defaultdict(float), defaultdict(int)
    for r in tr:
        k = short(r["Kernel_Name"])
        dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        calls[k] += 1
    total = sum(dur.values())

    ctr = defaultdict(lambda: defaultdict(float))   # kernel -> counter -> sum over the step
    ndisp = defaultdict(lambda: defaultdict(int))
    for path in a.pmc:
        rows = list(csv.DictReader(open(path)))
        # one row per (dispatch, counter): order by dispatch, then keep the last step
        rows = last_step_rows(rows, lambda r: int(r["Dispatch_Id"]))
        for r in rows:
            k, c = short(r["Kernel_Name"]), r["Counter_Name"]
            ctr[k][c] += float(r["Counter_Value"])
            ndisp[k][c] += 1

    def avg(k, c):
        n = ndisp[k].get(c, 0)
        return ctr[k][c] / n if n else None

    print(f"one step: GPU kernel time {total:.2f} ms, {sum(calls.values())} dispatches")
    hdr = f"{'ms':>7} {'%':>5} {'calls':>5} {'MFMA%':>6} {'LDSconf':>7} {'HBM_MiB':>8} {'GB/s':>6}  kernel"
    print(hdr)
    agg_bytes = 0.0
    for k, t in sorted(dur.items(), key=lambda kv: -kv[1])[:a.top]:
        mf = avg(k, "MfmaUtil")
        busy, grbm = ctr[k].get("SQ_VALU_MFMA_BUSY_CYCLES"), ctr[k].get("GRBM_GUI_ACTIVE")
        if mf is None and busy is not None and grbm:
            # busy cycles summed over SIMDs / (GPU-active cycles per XCD x 256 CUs x 4 SIMDs)
            mf = 100.0 * busy / (grbm / 8 * 256 * 4)
        bc, li = ctr[k].get("SQ_LDS_BANK_CONFLICT"), ctr[k].get("SQ_LDS_IDX_ACTIVE")
        conf = bc / li if bc is not None and li else None
        fb = ctr[k].get("FETCH_SIZE", 0.0) + ctr[k].get("WRITE_SIZE", 0.0)   # KiB over the step
        agg_bytes += fb
        bw = fb * 1024 / (t / 1e3) / 1e9 if t > 0 and fb else None
        fmt = lambda v, f: (f % v) if v is not None else "-"
        print(f"{t:7.2f} {100 * t / total:5.1f} {calls[k]:5d} {fmt(mf, '%6.1f'):>6} {fmt(conf, '%7.3f'):>7} "
              f"{fb / 1024:8.1f} {fmt(bw, '%6.0f'):>6}  {k}")
    all_b = sum(ctr[k].get("FETCH_SIZE", 0.0) + ctr[k].get("WRITE_SIZE", 0.0) for k in ctr)
    print(f"step HBM traffic {all_b / 1024 / 1024:.2f} GiB -> {all_b * 1024 / (total / 1e3) / 1e12:.2f} TB/s "
          f"averaged over the kernel time")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-stream timeline summary of one bench step from a rocprofv3 kernel trace: wall time of the
step, busy time per queue, the time both queues ran kernels at once, and the kernels of the side
queue with the main-queue kernels they overlapped.

    python tools/timeline.py run_kernel_trace.csv [--detail]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--detail", action="store_true")
    o = ap.parse_args()
    rows = list(csv.DictReader(open(o.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "synth_video" in r["Kernel_Name"]]
    step = rows[idx[-2]:idx[-1]]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    queues = {}
    for r in step:
        queues.setdefault(r["Queue_Id"], []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                                     r["Kernel_Name"].split("(")[0][:70]))
    print(f"step wall {(t1 - t0) / 1e6:.2f} ms, {len(step)} kernels, queues {sorted(queues)}")

    def union(iv):
        iv = sorted(iv)
        tot, cs, ce = 0, None, None
        for s, e, *_ in iv:
            if cs is None or s > ce:
                if cs is not None:
                    tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        return tot + ((ce - cs) if cs is not None else 0)

    busy = {q: union(v) for q, v in queues.items()}
    for q, v in queues.items():
        print(f"queue {q}: {len(v)} kernels, busy {busy[q] / 1e6:.2f} ms, kernel sum {sum(e - s for s, e, _ in v) / 1e6:.2f} ms")
    allb = union([x for v in queues.values() for x in v])
    print(f"any queue busy {allb / 1e6:.2f} ms; overlap {(sum(busy.values()) - allb) / 1e6:.2f} ms; "
          f"idle {(t1 - t0 - allb) / 1e6:.2f} ms")
    if o.detail and len(queues) > 1:
        qs = sorted(queues, key=lambda q: -len(queues[q]))
        main_q, side_q = qs[0], qs[1]
        for s, e, n in queues[side_q]:
            ov = [(max(s, ms), min(e, me), mn) for ms, me, mn in queues[main_q] if ms < e and me > s]
            print(f"{(s - t0) / 1e3:8.0f} {(e - s) / 1e3:7.0f} us  {n[:40]:40s} || " +
                  ", ".join(f"{mn[:28]}:{(b - a) / 1e3:.0f}" for a, b, mn in ov[:6]))


if __name__ == "__main__":
    main()

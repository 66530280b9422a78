#!/usr/bin/env python3
"""Write a committed profile summary (profiles/<name>.md) from a gpurun_out run:
bench JSON line, rocprofv3 per-kernel time per step, and the per-layer conv table.

    python tools/profile_summary.py NAME [--steps 5] [--stats gpurun_out/prof_bs256/run_kernel_stats.csv]
"""
import argparse
import csv
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--steps", type=float, default=5.0, help="profiled steps (warmup + timed) in the trace")
    ap.add_argument("--stats", default="gpurun_out/prof_bs256/run_kernel_stats.csv")
    ap.add_argument("--bench", default="gpurun_out/bench_bs256.json")
    ap.add_argument("--conv", default="gpurun_out/conv_bench.txt")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    out = [f"# Profile: {a.name}", ""]
    if os.path.exists(a.bench):
        line = [x for x in open(a.bench).read().splitlines() if x.startswith("{")]
        if line:
            b = json.loads(line[-1])
            out += ["## bench.py", "", "```json", json.dumps(b, indent=1), "```", ""]
    if os.path.exists(a.stats):
        rows = list(csv.DictReader(open(a.stats)))
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        out += [f"## rocprofv3 --kernel-trace --stats (per step, {a.steps:g} profiled steps)", "",
                f"Total GPU kernel time per step: **{tot / 1e6 / a.steps:.2f} ms** over {len(rows)} kernels.", "",
                "| ms/step | % | calls/step | avg µs | kernel |", "|---:|---:|---:|---:|---|"]
        for r in rows[:a.top]:
            t, c = float(r["TotalDurationNs"]), float(r["Calls"])
            name = r["Name"].replace("|", "\\|")
            if len(name) > 90:
                name = name[:90] + "…"
            out.append(f"| {t / 1e6 / a.steps:.2f} | {100 * t / tot:.1f} | {c / a.steps:.1f} | {t / c / 1e3:.1f} | `{name}` |")
        out.append("")
    if os.path.exists(a.conv):
        lines = [x for x in open(a.conv).read().splitlines() if not x.startswith("/opt")]
        out += ["## Per-layer conv kernels (tools/conv_bench.py, isolated, bs 256)", "", "```"] + lines + ["```", ""]
    os.makedirs("profiles", exist_ok=True)
    path = os.path.join("profiles", f"{a.name}.md")
    with open(path, "w") as f:
        f.write("\n".join(out))
    print(path)


if __name__ == "__main__":
    main()

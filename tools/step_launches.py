"""Launches per training step in a rocprofv3 kernel trace (steps delimited by adam_kernel):
python tools/step_launches.py run_kernel_trace.csv [--top N]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"].lower()]
    step = rows[ends[-2] + 1:ends[-1] + 1]
    queues = collections.Counter(r.get("Queue_Id", "") for r in step)
    print(f"launches in the last step: {len(step)}  per queue: {dict(queues)}")
    names = collections.Counter(r["Kernel_Name"].split("(")[0][:90] for r in step)
    short = sum(1 for r in step if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) < 10000)
    print(f"kernels < 10 us: {short}")
    for k, v in names.most_common(top):
        print(f"{v:5d}  {k}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-kernel time of one training step from a rocprofv3 kernel trace (steps delimited by adam_kernel).

usage: trace_breakdown.py <kernel_trace.csv> [step_index] [other_trace.csv]
With a second trace, prints both side by side (e.g. graph replay vs eager launches).
"""
import collections
import csv
import sys


def step_kernels(path, step):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [int(r["End_Timestamp"]) for r in rows if "adam_kernel" in r["Kernel_Name"]]
    lo, hi = ends[step - 1], ends[step]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        s = int(r["Start_Timestamp"])
        if lo < s <= hi:
            n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:56]
            agg[n][0] += 1
            agg[n][1] += (int(r["End_Timestamp"]) - s) / 1e3
    return agg


def main():
    a = step_kernels(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
    b = step_kernels(sys.argv[3], int(sys.argv[2]) if len(sys.argv) > 2 else 4) if len(sys.argv) > 3 else None
    keys = sorted(a, key=lambda k: -a[k][1])
    if b:
        keys += [k for k in b if k not in a]
    print(f"{'kernel':56} {'calls':>5} {'us':>9}" + (f" {'calls':>5} {'us':>9}" if b else ""))
    for k in keys:
        ca, ta = a.get(k, [0, 0.0])
        line = f"{k:56} {ca:5d} {ta:9.1f}"
        if b:
            cb, tb = b.get(k, [0, 0.0])
            line += f" {cb:5d} {tb:9.1f}"
        print(line)
    print(f"{'total':56} {'':5} {sum(v[1] for v in a.values()):9.1f}" +
          (f" {'':5} {sum(v[1] for v in b.values()):9.1f}" if b else ""))


if __name__ == "__main__":
    main()

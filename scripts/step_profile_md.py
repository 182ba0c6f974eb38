#!/usr/bin/env python3
"""Markdown summary of training steps from a rocprofv3 kernel trace (steps delimited by the starts of
the first layer's conv_first_kernel; the optimizer may end a step on two streams):
wall / per-queue busy / union busy per step, per-queue kernel totals of one step, and the main
queue's kernel sequence with the idle gap before each launch.

usage: step_profile_md.py <kernel_trace.csv> <title> [--sequence]
"""
import collections
import csv
import sys


def union(iv):
    iv = sorted(iv)
    tot, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + ce - cs


def main(path, title, sequence):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [int(r["Start_Timestamp"]) for r in rows if "conv_first_kernel" in r["Kernel_Name"]]
    print(f"# {title}\n")
    print(f"Source: rocprofv3 --kernel-trace (`{path.split('/')[-1]}`); a step starts at the first layer's conv.\n")
    print("## Per step (us)\n")
    print("| step | wall | union busy | " + " | ".join(f"queue {q} busy" for q in sorted({r['Queue_Id'] for r in rows})) + " | kernels |")
    qs = sorted({r["Queue_Id"] for r in rows})
    print("|---:|---:|---:|" + "---:|" * len(qs) + "---:|")
    steps = []
    for k in range(1, len(ends)):
        lo, hi = ends[k - 1], ends[k]
        st = [r for r in rows if lo <= int(r["Start_Timestamp"]) < hi]
        steps.append(st)
        busy = {q: sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in st if r["Queue_Id"] == q) / 1e3
                for q in qs}
        u = union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in st]) / 1e3
        print(f"| {k} | {(hi - lo) / 1e3:.1f} | {u:.1f} | " + " | ".join(f"{busy[q]:.1f}" for q in qs) + f" | {len(st)} |")
    st = steps[-2] if len(steps) > 1 else steps[-1]
    print("\n## Kernel totals of one step, per queue\n")
    for q in qs:
        agg = collections.defaultdict(lambda: [0, 0.0])
        for r in st:
            if r["Queue_Id"] != q:
                continue
            n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
            agg[n][0] += 1
            agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot = sum(v[1] for v in agg.values())
        print(f"queue {q}: {sum(v[0] for v in agg.values())} kernels, {tot:.1f} us\n")
        print("| kernel | calls | us | us / call |\n|---|---:|---:|---:|")
        for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
            print(f"| `{n}` | {c} | {t:.1f} | {t / c:.1f} |")
        print()
    for qq in (qs if sequence else []):
        print(f"## Queue {qq} sequence of one step\n\n```\n start us   gap us  dur us     grid kernel")
        t0 = int(st[0]["Start_Timestamp"])
        prev = None
        for r in st:
            if r["Queue_Id"] != qq:
                continue
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s - prev) / 1e3 if prev else 0.0
            prev = e
            print(f"{(s - t0) / 1e3:9.1f} {gap:8.1f} {(e - s) / 1e3:7.1f} {r['Grid_Size_X']:>8} "
                  f"{r['Kernel_Name'].split('(')[0].replace('void ', '')[:60]}")
        print("```")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], "--sequence" in sys.argv)

#!/usr/bin/env python3
"""Busy/idle accounting of the graph-replayed training step from a rocprofv3 kernel trace.

Steps are delimited by ``adam_kernel`` (one per step). For each step interval this prints the wall
span, the union of kernel execution intervals (GPU busy), the idle time between kernels, and the
summed kernel time (> busy when the wgrad side stream overlaps the main stream).
usage: graph_gaps.py <kernel_trace.csv>
"""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [int(r["End_Timestamp"]) for r in rows if "adam_kernel" in r["Kernel_Name"]]
    print(f"{'step':>4} {'wall ms':>8} {'busy ms':>8} {'idle ms':>8} {'sum ms':>8} {'kernels':>7}")
    for s in range(1, len(ends)):
        lo, hi = ends[s - 1], ends[s]
        ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
              if lo < int(r["Start_Timestamp"]) <= hi]
        busy, cur_s, cur_e = 0, None, None
        for a, b in ks:
            if cur_e is None or a > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = a, b
            else:
                cur_e = max(cur_e, b)
        if cur_e is not None:
            busy += cur_e - cur_s
        tot = sum(b - a for a, b in ks)
        print(f"{s:4d} {(hi - lo) / 1e6:8.3f} {busy / 1e6:8.3f} {(hi - lo - busy) / 1e6:8.3f} {tot / 1e6:8.3f} {len(ks):7d}")


if __name__ == "__main__":
    main(sys.argv[1])

#!/usr/bin/env python3
"""Gradient all-reduce / compute overlap in one training step, from a rocprofv3 kernel trace.

usage: comm_overlap.py <kernel_trace.csv> [step_index]

A step is delimited by consecutive ``adam_kernel`` ends (as in trace_breakdown.py). For every RCCL
kernel (name contains "nccl"/"rccl") in that step it prints its duration, how much of it ran while
at least one compute kernel was also executing, and the compute kernels it overlapped most (by
overlapped time) -- the evidence that the bucketed all-reduces run under the weight-gradient side
stream instead of after backward.
"""
import collections
import csv
import sys


def _is_comm(name: str) -> bool:
    n = name.lower()
    return "nccl" in n or "rccl" in n


def _short(name: str) -> str:
    return name.split("(")[0].replace("void ", "")[:60]


def main():
    path = sys.argv[1]
    step = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [int(r["End_Timestamp"]) for r in rows if "adam_kernel" in r["Kernel_Name"]]
    lo, hi = ends[step - 1], ends[step]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows
          if lo < int(r["Start_Timestamp"]) <= hi]
    comm = [k for k in ks if _is_comm(k[2])]
    comp = [k for k in ks if not _is_comm(k[2])]
    print(f"step {step}: {(hi - lo) / 1e3:.1f} us, {len(ks)} kernels, {len(comm)} RCCL kernels")
    tot = ovl_tot = 0.0
    print(f"{'RCCL kernel':<44} {'start_us':>9} {'dur_us':>8} {'overlap_us':>10}  top overlapped compute kernels")
    for s, e, n in comm:
        # union of compute intervals clipped to [s, e]
        iv = sorted((max(s, a), min(e, b)) for a, b, _ in comp if a < e and b > s)
        cov, cur_s, cur_e = 0, None, None
        for a, b in iv:
            if cur_e is None or a > cur_e:
                if cur_e is not None:
                    cov += cur_e - cur_s
                cur_s, cur_e = a, b
            else:
                cur_e = max(cur_e, b)
        if cur_e is not None:
            cov += cur_e - cur_s
        by = collections.defaultdict(int)
        for a, b, m in comp:
            if a < e and b > s:
                by[_short(m)] += min(e, b) - max(s, a)
        top = ", ".join(f"{k} {v / 1e3:.0f}us" for k, v in sorted(by.items(), key=lambda kv: -kv[1])[:3])
        d = (e - s) / 1e3
        tot += d
        ovl_tot += cov / 1e3
        print(f"{_short(n)[:44]:<44} {(s - lo) / 1e3:9.1f} {d:8.1f} {cov / 1e3:10.1f}  {top}")
    if comm:
        print(f"total RCCL kernel time {tot:.1f} us, overlapped with compute {ovl_tot:.1f} us "
              f"({100 * ovl_tot / max(tot, 1e-9):.0f} %)")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Kernel timeline of one serving-engine frame from a rocprofv3 kernel trace.

Frames are delimited by ``h2d_copy_kernel`` (the colour upload) or, without it, ``preprocess_kernel``. Prints, per kernel position of the
frame, the start offset and duration of the second-to-last complete frame plus the median duration
over the last (up to) 50 frames with the same kernel sequence, and the summed kernel time.
usage: serve_frame.py <kernel_trace.csv> [first_frame]
first_frame: take the reference frame and the median window from frames [first, first + 50) instead of
the last 50 (e.g. the sequential engine phase of bench_serve, before the pipelined frames overlap).
"""
import csv
import statistics
import sys


def main(path, first=None):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # a frame starts at its colour upload kernel where the runner uploads by kernel, else at the preprocess
    start_k = "h2d_copy_kernel" if any(r["Kernel_Name"].startswith("h2d_copy_kernel") for r in rows) else "preprocess_kernel"
    idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(start_k)]
    if len(idx) < 3:
        print("fewer than 3 frames in the trace")
        return
    frames = [rows[a:b] for a, b in zip(idx[:-1], idx[1:])]
    win = frames[-51:-1] if first is None else frames[first:first + 50]
    ref = win[-1]
    sig = [r["Kernel_Name"] for r in ref]
    same = [f for f in win if [r["Kernel_Name"] for r in f] == sig]
    t0 = int(ref[0]["Start_Timestamp"])
    tot = tmed = 0.0
    print(f"{'start us':>9} {'dur us':>7} {'med us':>7} {'grid':>8} kernel   (median over {len(same)} frames)")
    for k, r in enumerate(ref):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        med = statistics.median(int(f[k]["End_Timestamp"]) - int(f[k]["Start_Timestamp"]) for f in same) / 1e3
        tot += (e - s) / 1e3
        tmed += med
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {med:7.1f} {r['Grid_Size_X']:>8} "
              f"{r['Kernel_Name'].split('(')[0][:60]}")
    span = (int(ref[-1]["End_Timestamp"]) - t0) / 1e3
    print(f"kernel sum {tot:.1f} us (median-frame sum {tmed:.1f} us), first start -> last end {span:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)

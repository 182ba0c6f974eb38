#!/usr/bin/env python3
"""Kernel timeline of one serving-engine frame from a rocprofv3 kernel trace.

Frames are delimited by ``preprocess_kernel`` (one per frame); the second-to-last complete frame is
printed (start offset, duration, grid, kernel) with the summed kernel time.
usage: serve_frame.py <kernel_trace.csv>
"""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("preprocess_kernel")]
    if len(idx) < 3:
        print("fewer than 3 frames in the trace")
        return
    i0, i1 = idx[-3], idx[-2]
    t0 = int(rows[i0]["Start_Timestamp"])
    tot = 0
    print(f"{'start us':>9} {'dur us':>7} {'grid':>8} kernel")
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        tot += e - s
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {r['Grid_Size_X']:>8} {r['Kernel_Name'].split('(')[0][:60]}")
    print(f"kernel sum {tot / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])

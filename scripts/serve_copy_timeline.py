#!/usr/bin/env python3
"""One serving frame's device timeline -- kernels AND memory copies -- from a rocprofv3
--kernel-trace --memory-copy-trace run (scripts/gpu_serve_copies.sh): where the engine's GPU time
outside the kernels goes. Frames are delimited by preprocess_kernel; copies in the window from 80 us
before a frame's preprocess to the next frame's preprocess are attributed to it.
usage: serve_copy_timeline.py <dir with serve_kernel_trace.csv + serve_memory_copy_trace.csv> [frame]
"""
import csv
import os
import statistics
import sys


def main(d, frame=None):
    ks = sorted(csv.DictReader(open(os.path.join(d, "serve_kernel_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
    cs = sorted(csv.DictReader(open(os.path.join(d, "serve_memory_copy_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
    pre = [int(r["Start_Timestamp"]) for r in ks if r["Kernel_Name"].startswith("preprocess_kernel")]
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:48]) for r in ks]
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
            r["Direction"].replace("MEMORY_COPY_", "copy ") + f" (stream {r['Stream_Id']})") for r in cs]
    ev.sort()
    spans, lead, tail = [], [], []
    rows_of = {}
    for i in range(1, len(pre) - 1):
        a, b = pre[i] - 80_000, pre[i + 1] - 80_000
        fe = [e for e in ev if a <= e[0] < b]
        if not fe:
            continue
        first = min(e[0] for e in fe)
        last = max(e[1] for e in fe)
        spans.append((last - first) / 1e3)
        lead.append((pre[i] - first) / 1e3)
        kend = max(e[1] for e in fe if not e[2].startswith("copy"))
        tail.append((last - kend) / 1e3)
        rows_of[i] = fe
    k = frame if frame is not None else len(pre) // 3
    fe = rows_of.get(k) or next(iter(rows_of.values()))
    t0 = min(e[0] for e in fe)
    print(f"{'start us':>9} {'dur us':>7}  event   (frame {k})")
    for s, e, n in fe:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {n}")
    print(f"frames {len(spans)}: first event -> last event p50 {statistics.median(spans):.1f} us; "
          f"copies before the preprocess p50 {statistics.median(lead):.1f} us; after the last kernel p50 "
          f"{statistics.median(tail):.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)

#!/usr/bin/env python3
"""Dump the kernel dispatches of a rocprofv3 rocpd database (``-o run`` -> run_results.db) as
(start_us, dur_us, grid, name) rows in time order, optionally only the last ``--last`` dispatches,
and print a median-per-position sequence of the repeating unit that starts at ``--anchor`` (a kernel
name substring). Usage: rocpd_kernels.py DB [--anchor NAME] [--last N]"""
import argparse
import sqlite3
from collections import defaultdict

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--anchor", default="")
    ap.add_argument("--units", type=int, default=20)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    grid = "grid_x" if "grid_x" in cols else None
    q = f"select start, end, {name_col}, {grid if grid else 0} from kernels order by start"
    rows = db.execute(q).fetchall()
    t0 = rows[0][0]
    ks = [((s - t0) / 1e3, (e - s) / 1e3, g, n) for s, e, n, g in rows]
    if not a.anchor:
        for r in ks[-200:]:
            print(f"{r[0]:12.1f} {r[1]:8.1f} {r[2]:9} {r[3][:90]}")
        return
    starts = [i for i, r in enumerate(ks) if a.anchor in r[3]]
    units = [ks[starts[i]:starts[i + 1]] for i in range(len(starts) - 1)][-a.units:]
    L = min(len(u) for u in units)
    units = [u for u in units if len(u) == L] or units
    print(f"{len(units)} units of {L} kernels (anchor {a.anchor!r})")
    print(f"{'off us':>9} {'dur us':>8} {'grid':>9} kernel")
    for p in range(L):
        off = np.median([u[p][0] - u[0][0] for u in units])
        dur = np.median([u[p][1] for u in units])
        print(f"{off:9.1f} {dur:8.1f} {units[0][p][2]:9} {units[0][p][3][:100]}")
    span = np.median([u[-1][0] + u[-1][1] - u[0][0] for u in units])
    print(f"median unit span {span:.1f} us, kernel sum {np.median([sum(k[1] for k in u) for u in units]):.1f} us")


if __name__ == "__main__":
    main()

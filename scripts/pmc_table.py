#!/usr/bin/env python3
"""Per-dispatch PMC table (markdown) from rocprofv3 --pmc runs of the same program, one counter set per
run (<dir>/set*/pmc_counter_collection.csv). Dispatches are matched across the runs by their order
among the selected kernels; with --shapes (conv_microbench order) each kernel dispatch is labelled
with its layer shape (the microbench runs every shape twice: applicability check + timed rep).

usage: pmc_table.py <dir> [--match conv,wgrad] [--shapes fwd|wgrad] [--batch 64] [--every 2]

MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (256 CUs x 4 SIMDs x kernel cycles), kernel cycles =
GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs). HBM-side fetch = FETCH_SIZE (KB) / duration.
"""
import argparse
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def load(d, match):
    sets = []
    for f in sorted(glob.glob(os.path.join(d, "set*", "pmc_counter_collection.csv"))):
        acc = collections.OrderedDict()
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not any(m in name for m in match):
                continue
            k = int(r["Dispatch_Id"])
            e = acc.setdefault(k, {"name": name.split("(")[0].replace("void ", ""),
                                   "dur_us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                                   "grid": r.get("Grid_Size", "")})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        sets.append([acc[k] for k in sorted(acc)])
    n = min(len(s) for s in sets) if sets else 0
    out = []
    for i in range(n):
        m = {}
        for s in sets:
            for k, v in s[i].items():
                if k in ("dur_us",):
                    m.setdefault("durs", []).append(v)
                else:
                    m[k] = v
        m["dur_us"] = sorted(m.pop("durs"))[len(sets) // 2]
        out.append(m)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="conv,wgrad")
    ap.add_argument("--shapes", default=None, choices=[None, "fwd", "wgrad"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--every", type=int, default=2, help="dispatches per shape (microbench: check + timed)")
    ap.add_argument("--skip", default="reduce,group_sum", help="kernels left out of the table")
    a = ap.parse_args()
    rows = load(a.dir, a.match.split(","))
    skip = [s for s in a.skip.split(",") if s]
    rows = [r for r in rows if not any(s in r["name"] for s in skip)]
    labels = [""] * len(rows)
    if a.shapes:
        from conv_microbench import SHAPES
        for i in range(len(rows)):
            k = i // a.every
            if k < len(SHAPES):
                H, c1, c2, co = SHAPES[k]
                labels[i] = f"{a.batch}x{H}x{H} {c1}+{c2}->{co}"
        rows = rows[a.every - 1::a.every]
        labels = labels[a.every - 1::a.every]
    print("| kernel | shape | us | MFMA busy | VALU/MFMA | SALU/MFMA | LDS/MFMA | LDS bank confl. | "
          "L2 hit | fetch GB/s |")
    print("|---|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for r, lab in zip(rows, labels):
        mf = r.get("SQ_INSTS_MFMA", 0.0)
        cyc = r.get("GRBM_GUI_ACTIVE", 0.0) / 8
        busy = 100 * r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * cyc) if cyc else float("nan")
        per = (lambda c: f"{r.get(c, 0.0) / mf:.2f}" if mf else "-")
        hit, miss = r.get("TCC_HIT_sum"), r.get("TCC_MISS_sum")
        l2 = f"{100 * hit / (hit + miss):.0f} %" if hit is not None and (hit + miss) else "-"
        fetch = r.get("FETCH_SIZE")
        gbs = f"{fetch * 1024 / (r['dur_us'] * 1e-6) / 1e9:.0f}" if fetch is not None else "-"
        name = r["name"] if len(r["name"]) < 60 else r["name"][:57] + "..."
        print(f"| `{name}` | {lab} | {r['dur_us']:.1f} | {busy:.0f} % | {per('SQ_INSTS_VALU')} | "
              f"{per('SQ_INSTS_SALU')} | {per('SQ_INSTS_LDS')} | {r.get('SQ_LDS_BANK_CONFLICT', 0):.0f} | {l2} | {gbs} |")


if __name__ == "__main__":
    main()

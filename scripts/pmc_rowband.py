#!/usr/bin/env python3
"""Per-layer PMC table for `rowband_bench.py --variants 2,18` run under rocprofv3 --pmc, one counter set
per run (<dir>/set*/pmc_counter_collection.csv; sets as in scripts/pmc_sets_step.txt).

rowband_bench dispatches, per SHAPES entry, 1 check run + rounds x 2 x reps graph replays of each variant:
variant 2 = conv_igemm_kernel (+ its split-K reduce), variant 18 = conv_rowband_x_kernel. Dispatches are
assigned to shapes by their order; a reduce belongs to the igemm dispatch before it.

usage: pmc_rowband.py <dir> [--per-shape 21]
"""
import argparse
import collections
import csv
import glob
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def load_set(f):
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "igemm" in name:
            kind = "igemm"
        elif "splitk_reduce" in name:
            kind = "reduce"
        elif "rowband" in name:
            kind = "rowband"
        else:
            continue
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, {"kind": kind, "name": name.split("(")[0].replace("void ", ""),
                                "dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [disp[k] for k in sorted(disp)]


def by_shape(rows, per):
    """{shape index: {"v2": [(igemm, reduce|None)], "v18": [rowband]}}"""
    out = collections.defaultdict(lambda: {"v2": [], "v18": []})
    n_ig = n_rb = 0
    last = None
    for e in rows:
        if e["kind"] == "igemm":
            last = [e, None]
            out[n_ig // per]["v2"].append(last)
            n_ig += 1
        elif e["kind"] == "reduce" and last is not None:
            last[1] = e
        elif e["kind"] == "rowband":
            out[n_rb // per]["v18"].append(e)
            n_rb += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--per-shape", type=int, default=21)
    ap.add_argument("--batch", type=int, default=1)
    a = ap.parse_args()
    from rowband_bench import SHAPES
    sets = [by_shape(load_set(f), a.per_shape)
            for f in sorted(glob.glob(os.path.join(a.dir, "set*", "pmc_counter_collection.csv")))]

    def med(vals):
        vals = [v for v in vals if v is not None]
        return statistics.median(vals) if vals else None

    def stat(k, v, fn):
        return med([fn(x) for s in sets for x in s[k][v]])

    def ctr(e, c):
        return e.get(c) if e is not None else 0.0

    print("| layer | HxW | Cin->Cout | fused | kernel | us | HBM fetch MB | write MB | fetch GB/s | MFMA busy |")
    print("|---|---|---|---|---|---:|---:|---:|---:|---:|")
    tot = {"v2": 0.0, "v18": 0.0}
    for k, (name, H, C1, C2, Co, fuse) in enumerate(SHAPES):
        if not any(s[k]["v2"] or s[k]["v18"] for s in sets):
            continue
        for v in ("v2", "v18"):
            if v == "v2":
                dur = stat(k, v, lambda p: p[0]["dur"] + (p[1]["dur"] if p[1] else 0.0))
                fet = stat(k, v, lambda p: p[0].get("FETCH_SIZE") and p[0]["FETCH_SIZE"] + ctr(p[1], "FETCH_SIZE"))
                wr = stat(k, v, lambda p: p[0].get("WRITE_SIZE") and p[0]["WRITE_SIZE"] + ctr(p[1], "WRITE_SIZE"))
                busy = stat(k, v, lambda p: p[0].get("GRBM_GUI_ACTIVE") and
                            100 * p[0]["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * p[0]["GRBM_GUI_ACTIVE"] / 8))
                kern = "igemm<128,128,8> + split-K reduce" if any(
                    p[1] for s in sets for p in s[k][v]) else "igemm (no split)"
            else:
                dur = stat(k, v, lambda e: e["dur"])
                fet = stat(k, v, lambda e: e.get("FETCH_SIZE"))
                wr = stat(k, v, lambda e: e.get("WRITE_SIZE"))
                busy = stat(k, v, lambda e: e.get("GRBM_GUI_ACTIVE") and
                            100 * e["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * e["GRBM_GUI_ACTIVE"] / 8))
                names = {e["name"] for s in sets for e in s[k][v]}
                kern = ", ".join(sorted(n.replace("conv_rowband_x_kernel", "rowband_x") for n in names))
            if dur is None:
                continue
            tot[v] += dur
            f = lambda x, d=1: "-" if x is None else f"{x:.{d}f}"
            gbs = None if fet is None or not dur else fet * 1024 / (dur * 1e-6) / 1e9
            print(f"| {name} | {H}x{H} | {C1}{'+' + str(C2) if C2 else ''}->{Co} | {fuse or '-'} | {kern} | "
                  f"{dur:.1f} | {f(fet and fet / 1024, 2)} | {f(wr and wr / 1024, 2)} | {f(gbs, 0)} | "
                  f"{f(busy, 0)} % |")
    print(f"\nsum of per-dispatch median durations (under the profiler): v2 {tot['v2']:.1f} us, "
          f"v18 {tot['v18']:.1f} us")


if __name__ == "__main__":
    main()

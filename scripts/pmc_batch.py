#!/usr/bin/env python3
"""Summary of scripts/gpu_pmc_batch.sh: per batch size n, the dispatches of the last 100 batches (the timed
graph replays: after the 100th-from-last spline-fit launch, which ends every batch; before them the run
trains the model and captures the graphs), kernel time and MFMA busy per class.
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), as in profiles/rowband_pmc.md.

usage: pmc_batch.py <dir with n*/**/pmc_counter_collection.csv>
"""
import collections
import csv
import glob
import os
import sys


def load(f):
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, {"name": r["Kernel_Name"].split("(")[0].replace("void ", ""),
                                "dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [disp[k] for k in sorted(disp)]


def cls(name):
    if any(t in name for t in ("conv", "rowband", "splitk", "head", "upsample", "maxpool")):
        return "network (convs, upsamples, head)"
    if name.startswith("geo"):
        return "geometry"
    return "preprocess / JPEG / copies"


def main(root):
    print("| n | class | kernel us per frame | MFMA busy |")
    print("|---:|---|---:|---:|")
    for d in sorted(glob.glob(os.path.join(root, "n*"))):
        if not os.path.isdir(d):
            continue
        n = int(os.path.basename(d)[1:])
        fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not fs:
            continue
        ds = load(fs[0])
        fits = [i for i, e in enumerate(ds) if e["name"].startswith("geo_fit")]
        batches = 100
        ds = ds[fits[-batches - 1] + 1:fits[-1] + 1]
        agg = collections.defaultdict(lambda: [0.0, 0.0, 0.0])
        for e in ds:
            a = agg[cls(e["name"])]
            a[0] += e["dur"]
            a[1] += e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
            a[2] += 1024 * e.get("GRBM_GUI_ACTIVE", 0.0) / 8
        tot = [sum(v[i] for v in agg.values()) for i in range(3)]
        for c, v in sorted(agg.items()) + [("all", tot)]:
            busy = 100 * v[1] / v[2] if v[2] else 0.0
            print(f"| {n} | {c} | {v[0] / batches / n:.1f} | {busy:.1f} % |")


if __name__ == "__main__":
    main(sys.argv[1])

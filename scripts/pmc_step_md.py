#!/usr/bin/env python3
"""Per-kernel bytes and MFMA busy over ONE training step from rocprofv3 --pmc runs of bench.py
(scripts/gpu_pmc.sh with PMC_FILE=pmc_sets_step.txt: set1 FETCH_SIZE, set2 WRITE_SIZE, set3
SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE). A step = the dispatches from one conv_first_kernel to the
next (the last complete one of each run). The profiler serialises dispatches, so MFMA busy is each
kernel's own utilisation: busy cycles / (1,024 SIMDs x its cycles, GRBM_GUI_ACTIVE / 8 XCDs).

usage: pmc_step_md.py <pmc dir>
"""
import collections
import csv
import glob
import os
import sys


def step_dispatches(f):
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, {"name": r["Kernel_Name"].split("(")[0].replace("void ", ""),
                                "t": int(r["Start_Timestamp"]), "dur": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows = [disp[k] for k in sorted(disp)]
    firsts = [i for i, e in enumerate(rows) if e["name"].startswith("conv_first_kernel")]
    if len(firsts) < 2:
        return []
    a, b = firsts[-2], firsts[-1]
    return rows[a:b]


def main(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = {}
    for f in sorted(glob.glob(os.path.join(d, "set*", "pmc_counter_collection.csv"))):
        st = step_dispatches(f)
        cnt = collections.Counter(e["name"] for e in st)
        for e in st:
            g = agg[e["name"]]
            for c, v in e.items():
                if c in ("name", "t"):
                    continue
                if c == "dur":
                    g["dur_" + os.path.basename(os.path.dirname(f))] += v
                else:
                    g[c] += v
        for n, c in cnt.items():
            calls[n] = max(calls.get(n, 0), c)
    tf = sum(g.get("FETCH_SIZE", 0) for g in agg.values()) * 1024 / 1e9
    tw = sum(g.get("WRITE_SIZE", 0) for g in agg.values()) * 1024 / 1e9
    busy = sum(g.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for g in agg.values())
    cyc = sum(g.get("GRBM_GUI_ACTIVE", 0) for g in agg.values()) / 8
    mb = f"{100 * busy / (1024 * cyc):.0f} %" if cyc else "-"
    print(f"Per step: {tf:.1f} GB fetched + {tw:.1f} GB written; MFMA busy over the serialised kernel time {mb}\n")
    print("| kernel | calls | fetch GB | write GB | MFMA busy |")
    print("|---|---:|---:|---:|---:|")
    order = sorted(agg, key=lambda n: -(agg[n].get("FETCH_SIZE", 0) + agg[n].get("WRITE_SIZE", 0)))
    for n in order:
        g = agg[n]
        c = g.get("GRBM_GUI_ACTIVE", 0) / 8
        b = f"{100 * g.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (1024 * c):.0f} %" if c else "-"
        print(f"| `{n}` | {calls.get(n, 0)} | {g.get('FETCH_SIZE', 0) * 1024 / 1e9:.3f} | {g.get('WRITE_SIZE', 0) * 1024 / 1e9:.3f} | {b} |")


if __name__ == "__main__":
    main(sys.argv[1])

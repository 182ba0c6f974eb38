#!/usr/bin/env python3
"""Write profiles/conv_microbench.md from labelled conv_microbench.py JSON files.

usage: micro_report.py OUT.md LABEL=file.json [LABEL=file.json ...]
Every row is (layer shape, kind, column label); each column is one JSON file (one variant), so no
row is ever duplicated or left unlabelled.
"""
import json
import sys


def main():
    out = sys.argv[1]
    cols = []
    for arg in sys.argv[2:]:
        label, path = arg.split("=", 1)
        cols.append((label, json.load(open(path))))
    rows = {}
    for label, data in cols:
        for r in data:
            key = (r["shape"], r["kind"])
            tf = [v for k, v in r.items() if k.endswith("_tflops")]
            us = [v for k, v in r.items() if k.endswith("_us")]
            rows.setdefault(key, {})[label] = (tf[0] if tf else None, us[0] if us else None, r.get("splits"))
    md = ["# Conv kernels per U-Net layer shape (scripts/conv_microbench.py, one MI355X)", "",
          "TF/s = 2 * N * H * W * 9 * Cin * Cout / kernel time (median of interleaved rounds; wgrad times include",
          "the split-K slab reduction). Columns:", ""]
    for label, _ in cols:
        md.append(f"* **{label}**")
    md += ["", "| layer (N x H x W Cin1+Cin2 -> Cout) | kind | " + " | ".join(f"{l} TF/s (us)" for l, _ in cols) + " |",
           "|---|---|" + "---:|" * len(cols)]
    for (shape, kind), vals in rows.items():
        cells = []
        for label, _ in cols:
            v = vals.get(label)
            cells.append("" if v is None or v[0] is None else f"{v[0]:.1f} ({v[1]:.0f}{', ' + str(v[2]) + ' splits' if v[2] else ''})")
        md.append(f"| {shape} | {kind} | " + " | ".join(cells) + " |")
    open(out, "w").write("\n".join(md) + "\n")
    print("wrote", out)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Standalone time of the weight re-layout launch (csrc/optim.hip wprep_kernel) for the U-Net tables:
the dgrad layouts rebuilt on the side stream after Adam (bwd), and the whole table (all).

usage: python scripts/wprep_bench.py [--reps 50] [--decoder bilinear|transposed]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from robotic_discovery_platform_amd.models.unet import UNetNative  # noqa: E402
from robotic_discovery_platform_amd.ops import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--decoder", default="bilinear")
    a = ap.parse_args()
    C = native()
    dev = torch.device("cuda", 0)
    m = UNetNative(3, 1, bilinear=a.decoder == "bilinear", device=dev)
    st = m.store
    tables = {"bwd": (m._segs_bwd, m._nseg_bwd, m._wblk_bwd), "all": (m._segs, m._nseg, m._wblk)}
    out = {}
    for name, (segs, nseg, blk) in tables.items():
        for _ in range(3):
            C.wprep(st.flat, m.derived, segs, nseg, None, blk)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                C.wprep(st.flat, m.derived, segs, nseg, None, blk)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000.0 / a.reps)
        out[f"us_{name}"] = round(statistics.median(ts), 2)
        out[f"grid_{name}"] = int(blk)
    out["params"] = int(st.numel)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

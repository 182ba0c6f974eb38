#!/usr/bin/env python3
"""Serving network cost vs batch: the eval U-Net (BN folded, head + threshold fused) at N = 1, 2, 4, 8
frames per launch, captured in a hipGraph and replayed back to back; device ms per replay and per frame.

usage: python scripts/serve_batch_probe.py [--sizes 1,2,4,8] [--reps 200]
Decides whether batching concurrent streams' frames into one network launch pays (serve/engine.py).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = UNetNative(3, 1, device=dev, init_from=UNetRef(3, 1))
    hw, hb = m.store.view("outc.conv.weight").reshape(-1), m.store.view("outc.conv.bias")
    out = {}
    s = torch.cuda.Stream()
    for n in [int(v) for v in a.sizes.split(",")]:
        ex = m.executor(n, 256, 256, training=False)
        ex.set_input(torch.rand(n, 3, 256, 256, device=dev))
        mask = torch.empty(n * 256 * 256, dtype=torch.uint8, device=dev)
        with torch.cuda.stream(s):
            ex.prepare_eval()
            ex.forward(head=False, refresh_eval=False, mask_head=(hw, hb, 0.0, mask))
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            ex.forward(head=False, refresh_eval=False, mask_head=(hw, hb, 0.0, mask))
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(a.reps):
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        med = ts[len(ts) // 2]
        out[n] = {"ms_per_launch": round(med, 4), "ms_per_frame": round(med / n, 4)}
        print(json.dumps({"N": n, **out[n]}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""BatchEngine (serve/engine.py) device time per batch size: n frames forced into one batch (all n
positions taken before staging), repeated; reports the GPU time per batch (upload + graph) and per frame,
and the same for the single-frame pipeline (FramePipeline). ``--src jpeg`` uses encoded requests.
Used for profiles/serve_batch.md (run under rocprofv3 --kernel-trace for the per-kernel split)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--src", choices=["bgr", "jpeg"], default="bgr")
    ap.add_argument("--sizes", default="1,2,3,4")
    ap.add_argument("--single", type=int, default=1, help="0: skip the single-frame pipeline (PMC runs)")
    a = ap.parse_args()
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K
    from robotic_discovery_platform_amd.serve.bench_serve import prepare_model
    from robotic_discovery_platform_amd.serve.client import make_request
    from robotic_discovery_platform_amd.serve.engine import SRC_BGR, SRC_JPEG, BatchEngine, FramePipeline
    dev = torch.device("cuda")
    model, scenes = prepare_model(dev, 30, n_scenes=8)
    out = {}
    if a.single:
        single = FramePipeline(model, DEFAULT_K, 0.001, graph=True)
        g = []
        for i in range(a.reps):
            sc = scenes[i % 8]
            g.append(single.process(sc.color, sc.depth).timings["gpu_ms"])
        out["single_gpu_ms_p50"] = round(float(np.median(g)), 4)
    src = SRC_JPEG if a.src == "jpeg" else SRC_BGR
    reqs = [make_request(sc.color, sc.depth) for sc in scenes] if src == SRC_JPEG else None
    be = BatchEngine(model, DEFAULT_K, 0.001, src=src, positions=4, window_us=1e6)
    for n in [int(x) for x in a.sizes.split(",")]:
        gm, wall = [], []
        for r in range(a.reps):
            t0 = time.perf_counter()
            pos = [be._acquire() for _ in range(n)]
            tk = []
            for i, p in enumerate(pos):
                if src == SRC_JPEG:
                    rq = reqs[(r + i) % 8]
                    tk.append(be.submit_encoded(rq.color_image.data, rq.depth_image.data, pos=p)[1])
                else:
                    sc = scenes[(r + i) % 8]
                    tk.append(be.submit(sc.color, sc.depth, pos=p))
            res = [be.collect_encoded(t) if src == SRC_JPEG else be.collect(t) for t in tk]
            wall.append((time.perf_counter() - t0) * 1e3)
            gm.append(res[0].gpu_ms if src == SRC_JPEG else res[0].timings["gpu_ms"])
        out[f"batch{n}_gpu_ms_p50"] = round(float(np.median(gm)), 4)
        out[f"batch{n}_gpu_ms_per_frame"] = round(float(np.median(gm)) / n, 4)
        out[f"batch{n}_wall_ms_p50"] = round(float(np.median(wall)), 4)
        print(f"[batch] n={n}: {out}", file=sys.stderr, flush=True)
    be.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

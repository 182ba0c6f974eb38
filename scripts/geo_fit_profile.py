#!/usr/bin/env python3
"""Phase profile of the on-device spline fit on realistic serving frames.

Trains the serving model like bench_serve (default 200 steps), runs frames through the engine,
then re-launches the sort + fit on that frame's binned edge points with the kernel's phase
stamps enabled (geo_spline dbg=) and prints, per frame, m, iteration counts and microseconds per
phase. JSON lines to stdout.
"""
import argparse
import json
import sys

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--train-steps", type=int, default=200)
    ap.add_argument("--frames", type=int, default=8)
    a = ap.parse_args()
    sys.path.insert(0, ".")
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K
    from robotic_discovery_platform_amd.serve.bench_serve import prepare_model
    from robotic_discovery_platform_amd.serve.engine import FramePipeline
    dev = torch.device("cuda")
    model, scenes = prepare_model(dev, a.train_steps)
    p = FramePipeline(model, DEFAULT_K, 0.001, graph=True)
    g = p.geo
    c = g.cfg
    names = ["m", "lsq_iters", "smooth_iters", "total", "setup", "gram", "chol_lsq", "resid_lsq", "control", "btb",
             "chol_smooth", "resid_smooth", "eval", "n", "ev_deriv", "ev_samples", "ev_kappa", "ev_reduce", "ev_write"]
    for i in range(a.frames):
        sc = scenes[i % len(scenes)]
        r = p.process(sc.color, sc.depth)
        dbg = torch.zeros(20, dtype=torch.float64, device=dev)
        for _ in range(2):  # second run: warm
            g.C.geo_spline(g.out, g.kout, g.npts, g.sorted, g.gperm, g.u, g.res, c.smoothing, c.spline_degree,
                           c.num_samples, c.deriv_eps, c.min_points, c.min_edge_points, g.cov, dbg)
        torch.cuda.synchronize()
        d = dbg.cpu().tolist()
        out = {k: (int(v) if j in (0, 1, 2, 13) else round(v / 100.0, 2)) for j, (k, v) in enumerate(zip(names, d))}
        out["status"] = r.curvature.status
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

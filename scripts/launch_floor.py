#!/usr/bin/env python3
"""Per-kernel cost floor inside a replayed hipGraph on this GPU (what a fused-away launch saves).

Captures K back-to-back launches of (a) a 1-element torch fill, (b) the native maxpool on a tiny
and on the serving-size tensor, (c) a native 3x3 conv at 16^2 x 512 -> 512 without split-K, and
times graph replays with events; prints us per launch. JSON to stdout.
"""
import json
import sys

import torch


def per_launch(fn, k=200, reps=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(k):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * k)


def main():
    sys.path.insert(0, ".")
    from robotic_discovery_platform_amd.ops import native
    C = native()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    out = {}
    t = torch.zeros(1, device=dev)
    out["torch_fill_1elem"] = per_launch(lambda: t.fill_(1.0))
    xs = torch.zeros(1, 4, 4, 64, dtype=bf, device=dev)
    ys = torch.zeros(1, 2, 2, 64, dtype=bf, device=dev)
    out["maxpool_4x4x64"] = per_launch(lambda: C.maxpool2_fwd(xs, ys))
    xb = torch.randn(1, 32, 32, 512, device=dev).to(bf)
    yb = torch.zeros(1, 16, 16, 512, dtype=bf, device=dev)
    out["maxpool_32x32x512"] = per_launch(lambda: C.maxpool2_fwd(xb, yb))
    xc = torch.randn(1, 16, 16, 512, device=dev).to(bf)
    wc = (torch.randn(512, 9 * 512, device=dev) * 0.02).to(bf)
    yc = torch.zeros(1, 16, 16, 512, dtype=bf, device=dev)
    out["conv_16x16x512_nosplit"] = per_launch(lambda: C.conv_fwd(xc, None, wc, 9, 0, yc, None, None, 0, None, 0),
                                               k=50)
    n_ws = C.conv_ws_elems(1, 16, 16, 512, 0, 512, 9, 0, 0)
    ws = torch.zeros(n_ws, device=dev)
    out["conv_16x16x512_splitk_pair"] = per_launch(
        lambda: C.conv_fwd(xc, None, wc, 9, 0, yc, None, None, 0, None, 0, ws), k=50)
    print(json.dumps({k: round(v, 2) for k, v in out.items()}))


if __name__ == "__main__":
    main()

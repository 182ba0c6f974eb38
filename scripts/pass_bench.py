#!/usr/bin/env python3
"""Standalone rate of the memory-bound passes of the training step at their bs-64 shapes (the layers
where they are largest): BN apply (+ pool), BN backward reduce / apply, maxpool backward + BN reduce,
bilinear x2 upsample forward / backward (+ BN reduce), the training head forward / BN-backward apply. Median of interleaved rounds; GB/s = the bytes
each pass must move (tensor reads + writes) / time.

usage: python scripts/pass_bench.py [--batch 64] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robotic_discovery_platform_amd.ops import native  # noqa: E402


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    C = native()
    dev = "cuda"
    N = a.batch
    bf = torch.bfloat16

    def t(h, w, c):
        return torch.randn(N, h, w, c, device=dev).to(bf)

    def coef(c):
        return torch.cat([torch.zeros(c, device=dev), torch.ones(c, device=dev), torch.rand(c, device=dev) + 0.5,
                          torch.randn(c, device=dev) * 0.1]).contiguous()

    cases = []
    for (H, Cc) in ((256, 64), (128, 128), (64, 256)):
        y, out, da, dy = t(H, H, Cc), t(H, H, Cc), t(H, H, Cc), t(H, H, Cc)
        cf, c2 = coef(Cc), torch.randn(3 * Cc, device=dev)
        part = torch.zeros(1024 * 2 * Cc, device=dev)
        pool = t(H // 2, H // 2, Cc)
        dp = t(H // 2, H // 2, Cc)
        E = N * H * H * Cc * 2  # bytes of one full-resolution tensor
        cases += [
            (f"bn_relu_apply {H}^2 x {Cc}", 2 * E, lambda y=y, out=out, cf=cf: C.bn_relu_apply(y, out, cf, 1)),
            (f"bn_relu_apply_pool {H}^2 x {Cc}", 2 * E + E // 4,
             lambda y=y, out=out, pool=pool, cf=cf: C.bn_relu_apply_pool(y, out, pool, cf)),
            (f"bn_relu_bwd_reduce {H}^2 x {Cc}", 2 * E,
             lambda da=da, y=y, cf=cf, part=part: C.bn_relu_bwd_reduce(da, y, cf, 1, part)),
            (f"bn_relu_bwd_apply {H}^2 x {Cc}", 3 * E,
             lambda da=da, y=y, cf=cf, c2=c2, dy=dy: C.bn_relu_bwd_apply(da, y, cf, c2, dy, 1)),
            (f"maxpool2_bwd_bn_reduce {H}^2 x {Cc}", 3 * E + E // 4,
             lambda dp=dp, y=y, da=da, out=out, dy=dy, cf=cf, part=part: C.maxpool2_bwd_bn_reduce(dp, out, da, dy, y, cf, part)),
        ]
    for (h, Cc) in ((128, 64), (64, 128), (32, 256)):
        x, u = t(h, h, Cc), t(2 * h, 2 * h, Cc)
        ylow, cf = t(h, h, Cc), coef(Cc)
        dx = t(h, h, Cc)
        part = torch.zeros(4096 * 2 * Cc, device=dev)
        El = N * h * h * Cc * 2
        cases += [
            (f"upsample2_fwd {h}^2 -> {2 * h}^2 x {Cc}", El + 4 * El, lambda x=x, u=u: C.upsample2_fwd(x, u, 0, 0)),
            (f"upsample2_bwd + BN reduce {2 * h}^2 -> {h}^2 x {Cc}", 4 * El + 2 * El,
             lambda u=u, dx=dx, ylow=ylow, cf=cf, part=part: C.upsample2_bwd(u, dx, 0, 0, ylow, cf, part)),
        ]
    # the training head (last conv's BN + ReLU, 1x1 conv, BCE partials and the backward partials from
    # the same read of y; head_fwd GRAD) and its BN-backward apply (y read again, dy written)
    H, Cc = 256, 64
    M = N * H * H
    y = t(H, H, Cc)
    cf = coef(Cc)
    wt, b = torch.randn(64, device=dev) * 0.1, torch.randn(1, device=dev) * 0.1
    tg = (torch.rand(M, device=dev) > 0.5).float()
    nb = C.head_partial_blocks(M)
    lg, part = torch.zeros(M, device=dev), torch.zeros(nb * 65, device=dev)
    sums, loss = torch.zeros(4, device=dev), torch.zeros(2, device=dev)
    gp, bp = torch.zeros(nb * 65, device=dev), torch.zeros(nb * 128, device=dev)
    c2 = torch.randn(3 * Cc, device=dev)
    dyh = t(H, H, Cc)
    E = M * Cc * 2
    cases += [
        (f"head_fwd (BN, grad partials) {H}^2 x {Cc}", E + 8 * M,
         lambda: C.head_fwd(y, wt, b, tg, lg, part, sums, loss, 0.0, 1.0, cf, gp, bp, 1.0)),
        (f"head_bn_bwd_apply {H}^2 x {Cc}", 2 * E + 8 * M,
         lambda: C.head_bn_bwd_apply(y, wt, lg, tg, sums, cf, c2, dyh, 0.0, 1.0, 1.0)),
    ]
    for name, nbytes, fn in cases:
        fn()
    torch.cuda.synchronize()
    times = {name: [] for name, _, _ in cases}
    for _ in range(a.rounds):
        for name, _, fn in cases:
            times[name].append(timed(fn, a.reps))
    for name, nbytes, _ in cases:
        ms = statistics.median(times[name])
        print(json.dumps({"pass": name, "us": round(ms * 1e3, 1), "GB": round(nbytes / 1e9, 3),
                          "TB_per_s": round(nbytes / ms / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()

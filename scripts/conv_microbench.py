#!/usr/bin/env python3
"""A/B microbenchmark of conv kernel variants on the U-Net's layer shapes (one process, interleaved).

usage: python scripts/conv_microbench.py [--batch 32] [--variants 0,1] [--reps 10] [--wgrad]
Prints TF/s per (layer, variant): median over interleaved rounds (cdna_hip_programming.md §5.4 r24).
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robotic_discovery_platform_amd.ops import native  # noqa: E402

SHAPES = [  # (H, Cin1, Cin2, Cout)   spatial = H x H
    (256, 64, 0, 64), (128, 64, 0, 128), (128, 128, 0, 128), (64, 256, 0, 256), (32, 512, 0, 512),
    (16, 512, 0, 512), (32, 512, 512, 256), (64, 256, 256, 128), (128, 128, 128, 64), (256, 64, 64, 64),
    (128, 128, 0, 64), (64, 128, 0, 256), (32, 256, 0, 512), (32, 1024, 0, 512), (64, 512, 0, 256),
    (32, 512, 0, 256), (64, 256, 0, 128), (128, 64, 0, 128),
    (32, 512, 0, 1024), (64, 256, 0, 512), (16, 512, 0, 1024),  # dgrads of the Up convs' concat inputs
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--wgrad", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--halo-slab", type=int, default=1, help="wgrad: slab for the halo kernel's full split count")
    ap.add_argument("--shapes", default=None, help="comma list of shape indices")
    ap.add_argument("--ws", type=int, default=0, help="fwd: pass a split-K workspace (the training step has one)")
    ap.add_argument("--wgrad-blocks", type=int, default=2048,
                    help="split-K grid target of the generic wgrad kernel (the training step uses 512)")
    a = ap.parse_args()
    C = native()
    dev = torch.device("cuda")
    variants = [int(v) for v in a.variants.split(",")]
    results = []
    shapes = SHAPES if a.shapes is None else [SHAPES[int(i)] for i in a.shapes.split(",")]
    for (H, C1, C2, Co) in shapes:
        N = a.batch
        x1 = torch.randn(N, H, H, C1, device=dev).to(torch.bfloat16)
        x2 = torch.randn(N, H, H, C2, device=dev).to(torch.bfloat16) if C2 else None
        Cin = C1 + C2
        w = (torch.randn(Co, 9 * Cin, device=dev) * 0.02).to(torch.bfloat16)
        y = torch.empty(N, H, H, Co, dtype=torch.bfloat16, device=dev)
        stats = torch.zeros(max(C.conv_stats_rows(N * H * H, Co, 0), 1024) * 2 * Co, device=dev)
        flops = 2.0 * N * H * H * 9 * Cin * Co
        times = {v: [] for v in variants}
        ws = None
        if a.ws and not a.wgrad:
            n_ws = max(C.conv_ws_elems(N, H, H, C1, C2, Co, 9, 0, v) for v in variants)
            ws = torch.zeros(max(n_ws, 1), device=dev) if n_ws else None
        if a.wgrad:
            dy = torch.randn(N, H, H, Co, device=dev).to(torch.bfloat16)
            tiles = ((9 * Cin + 255) // 256) * (Co // 64)
            splits = max(1, min((a.wgrad_blocks + tiles - 1) // tiles, N * H * H // 2048))
            # sized for the halo kernel's own full-occupancy split choice too (the training step gives it
            # less on purpose: csrc/conv_wgrad.hip rdp_conv_wgrad_slab_elems)
            slab = torch.zeros(max(C.wgrad_slab_elems(N, H, H, Cin, Co, 9, 0, splits),
                                   C.wgrad_halo_slab_elems(N, H, H, Cin, Co) if a.halo_slab else 0), device=dev)
            out = torch.zeros(Co * 9 * Cin, device=dev)

        # v = 9: the BN-on-input row-ring path (x1 = producer's pre-BN y; 64 -> 64 at W % 64 == 0)
        # ([mean | invstd | scale | shift] of the producer's BN)
        coef = torch.cat([torch.zeros(2 * C1, device=dev), torch.rand(C1, device=dev) + 0.5,
                          torch.randn(C1, device=dev) * 0.1]).float()

        a_st = torch.empty_like(x1)

        def run(v):
            if a.wgrad:  # v = variant (0 auto, 4 generic, 5 halo)
                C.conv_wgrad(x1, x2, dy, 9, 0, 0, slab, out, 0, splits, v)
            elif v in (9, 10):  # 10: BN-on-input forward that also stores the activation
                if C.conv_fwd_bnin(x1, w, y, stats, coef, a_st if v == 10 else None) <= 0:
                    raise RuntimeError("bnin n/a")
            else:
                # v = bm_pref (1 halo, 2 igemm 128x128 8-wave, 4 / 5 ping-pong, 7 / 8 split-K ping-pong)
                C.conv_fwd(x1, x2, w, 9, 0, y, None, stats, v, None, 0, ws)

        ok = []
        for v in variants:  # a variant that does not apply to this shape (-1) is skipped
            try:
                run(v)
                ok.append(v)
            except RuntimeError:
                pass
        variants_s = ok
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for v in variants_s:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    run(v)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / a.reps)
        row = {"shape": f"{N}x{H}x{H} {C1}+{C2}->{Co}", "kind": "wgrad" if a.wgrad else "fwd"}
        if a.wgrad:
            row["splits"] = splits
            row["wgrad_blocks"] = a.wgrad_blocks
        for v in variants_s:
            med = statistics.median(times[v])
            row[f"v{v}_us"] = round(med * 1e3, 1)
            row[f"v{v}_tflops"] = round(flops / (med * 1e-3) / 1e12, 1)
        results.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        json.dump(results, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()

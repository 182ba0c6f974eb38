#!/usr/bin/env python3
"""Serving-size eval convs (BN folded + ReLU, N = 1): the row-band kernel (bm_pref 16,
csrc/conv_rowband.hip) against the split-K implicit GEMM + reduce launch pair (bm_pref 2: the 8-wave
128 x 128 kernel the auto dispatch otherwise picks at these shapes).

Each variant runs `--reps` convs back to back inside one captured hipGraph (kernel boundaries included,
as in the serving frame's graph); device time per conv = replay time / reps, median over interleaved
rounds. usage: python scripts/rowband_bench.py [--batch 1] [--reps 20] [--rounds 7]
"""
import argparse
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robotic_discovery_platform_amd.ops import native  # noqa: E402

# (name, H, C1, C2, Cout, fused output): the U-Net levels at <= 64^2 of a 256^2 frame
SHAPES = [("down2.conv1", 64, 128, 0, 256, None), ("down2.conv2", 64, 256, 0, 256, "pool"),
          ("down3.conv1", 32, 256, 0, 512, None), ("down3.conv2", 32, 512, 0, 512, "pool"),
          ("down4.conv1", 16, 512, 0, 512, None), ("down4.conv2", 16, 512, 0, 512, "up"),
          ("up1.conv1", 32, 512, 512, 512, None), ("up1.conv2", 32, 512, 0, 256, "up"),
          ("up2.conv1", 64, 256, 256, 256, None), ("up2.conv2", 64, 256, 0, 128, "up"),
          ("up3.conv1", 128, 128, 128, 128, None), ("down1.conv1", 128, 64, 0, 128, None),
          ("down1.conv2", 128, 128, 0, 128, "pool"), ("up3.conv2", 128, 128, 0, 64, "up")]


def frag_weights(w):
    """OHWI [Cout][9 Cin] -> the row-band kernel's fragment-major layout [Cout/16][9 Cin/32][64 lanes][8]
    (lane = 16 * (8-channel group) + row): every MFMA A fragment is 1 KiB contiguous."""
    co, k = w.shape
    return w.view(co // 16, 16, k // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().view(co, k)


def chain_bench(C, a):
    """--chain: the 16^2 level (down4 conv1 -> conv2, 512 -> 512 -> 512) as two row-band launches vs one
    persistent chain launch (conv_rowband_chain: row readiness counters, no kernel boundary) vs the split-K
    pair; outputs of the chain bitwise those of the launches."""
    dev = torch.device("cuda")
    N, H, Cs = a.batch, 16, [512, 512, 512]
    torch.manual_seed(0)
    x = torch.randn(N, H, H, Cs[0], device=dev).to(torch.bfloat16)
    ws, coefs, ys, ys2 = [], [], [], []
    for l in range(a.chain_layers):
        ci, co = Cs[min(l, 2)], Cs[min(l + 1, 2)]
        ws.append((torch.randn(co, 9 * ci, device=dev) / math.sqrt(9 * ci)).to(torch.bfloat16))
        cf = torch.zeros(4 * co, device=dev)
        C.bn_eval_coef(torch.rand(co, device=dev) + 0.5, torch.randn(co, device=dev) * 0.1, torch.zeros(co, device=dev),
                       torch.ones(co, device=dev), 1e-5, cf)
        coefs.append(cf)
        ys.append(torch.empty(N, H, H, co, dtype=torch.bfloat16, device=dev))
        ys2.append(torch.empty(N, H, H, co, dtype=torch.bfloat16, device=dev))
    cnt = torch.zeros(1 + len(ws) * N * H, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    kws = torch.zeros(max(max(C.conv_ws_elems(N, H, H, 512, 0, 512, 9, 0, 2), 1), 1), device=dev)

    def per_layer(pref):
        inp = x
        for w, y, cf in zip(ws, ys2, coefs):
            C.conv_fwd(inp, None, w, 9, 0, y, None, None, pref, cf, 1, kws)
            inp = y

    def chain():
        assert C.conv_rowband_chain(x, ws, ys, coefs, cnt, err)

    s = torch.cuda.Stream()
    runs = {"rowband_launches": lambda: per_layer(16), "chain": chain, "splitk_pairs": lambda: per_layer(2)}
    graphs = {}
    for k, fn in runs.items():
        with torch.cuda.stream(s):
            fn()
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(a.reps):
                fn()
        graphs[k] = g
    per_layer(16)
    chain()
    torch.cuda.synchronize()
    same = all(torch.equal(p, q) for p, q in zip(ys, ys2))
    times = {k: [] for k in runs}
    for _ in range(a.rounds):
        for k, g in graphs.items():
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1000.0 / a.reps)
    print(json.dumps({"chain_layers": len(ws), "N": N, "map": f"{H}x{H}", "bitwise_equal": same,
                      "err": int(err.item()), **{f"us_{k}": round(statistics.median(v), 2) for k, v in times.items()}}),
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chain", type=int, default=0, help="also time the persistent chain of the 16^2 level")
    ap.add_argument("--chain-layers", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--variants", default="2,16")
    a = ap.parse_args()
    C = native()
    if a.chain:
        chain_bench(C, a)
        return
    dev = torch.device("cuda")
    N = a.batch
    variants = [int(v) for v in a.variants.split(",")]
    total = {v: 0.0 for v in variants}
    s = torch.cuda.Stream()
    for (name, H, C1, C2, Co, fuse) in SHAPES:
        torch.manual_seed(0)
        x1 = torch.randn(N, H, H, C1, device=dev).to(torch.bfloat16)
        x2 = torch.randn(N, H, H, C2, device=dev).to(torch.bfloat16) if C2 else None
        Cin = C1 + C2
        w = (torch.randn(Co, 9 * Cin, device=dev) / math.sqrt(9 * Cin)).to(torch.bfloat16)
        coef = torch.zeros(4 * Co, device=dev)
        C.bn_eval_coef(torch.rand(Co, device=dev) + 0.5, torch.randn(Co, device=dev) * 0.1,
                       torch.zeros(Co, device=dev), torch.ones(Co, device=dev), 1e-5, coef)
        y = torch.empty(N, H, H, Co, dtype=torch.bfloat16, device=dev)
        pool = torch.empty(N, H // 2, H // 2, Co, dtype=torch.bfloat16, device=dev) if fuse == "pool" else None
        up = torch.empty(N, 2 * H, 2 * H, Co, dtype=torch.bfloat16, device=dev) if fuse == "up" else None
        n_ws = max([C.conv_ws_elems(N, H, H, C1, C2, Co, 9, 0, v) for v in variants if v < 17] + [1])
        ws = torch.zeros(max(n_ws, 1), device=dev)
        graphs = {}
        wf = frag_weights(w)
        for v in variants:
            if v == 18 and (Cin // 32) % 8 and Cin not in (64, 128):  # staged: 2, 4 or 8k chunks of 32 channels
                continue
            def run(v=v):
                if v in (17, 18):  # the row-band kernel on fragment-major weights (18: activation-staged)
                    if C.conv_rowband(x1, x2, wf, y, coef, pool, v - 16) < 0:
                        raise RuntimeError("conv_rowband: shape not taken")
                    return
                C.conv_fwd(x1, x2, w, 9, 0, y, None, None, v, coef, 1, ws, pool, up, 0, 0)
            try:
                with torch.cuda.stream(s):
                    run()
                s.synchronize()
            except RuntimeError:  # the variant does not take this shape
                continue
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(a.reps):
                    run()
            graphs[v] = g
        times = {v: [] for v in graphs}
        for _ in range(a.rounds):
            for v in graphs:
                graphs[v].replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                graphs[v].replay()
                e1.record()
                e1.synchronize()
                times[v].append(e0.elapsed_time(e1) * 1000.0 / a.reps)
        row = {"layer": name, "H": H, "cin": Cin, "cout": Co, "fused": fuse}
        for v in graphs:
            t = statistics.median(times[v])
            row[f"us_v{v}"] = round(t, 2)
            total[v] += t
        print(json.dumps(row), flush=True)
    print(json.dumps({"total_us": {f"v{v}": round(t, 1) for v, t in total.items()}}), flush=True)


if __name__ == "__main__":
    main()

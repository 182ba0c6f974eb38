#!/usr/bin/env python3
"""Library-GEMM reference for the deep U-Net convs: torch.matmul (hipBLASLt) on the plain GEMM with
the same M x N x K as each implicit-GEMM conv (M = N*H*W pixels, N = Cout, K = 9*Cin), bf16 in, bf16
out, random operands, next to this repo's conv kernel on the real conv (scripts/conv_microbench.py
shapes, auto dispatch). Median of interleaved rounds; TF/s = 2*M*N*K / time.

usage: python scripts/gemm_ceiling.py [--batch 64] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robotic_discovery_platform_amd.ops import native  # noqa: E402

SHAPES = [(64, 256, 256), (32, 512, 512), (32, 1024, 512), (64, 512, 256), (16, 512, 512), (128, 128, 128),
          (32, 256, 512), (64, 128, 256)]  # (H, Cin, Cout)


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
    ap.add_argument("--conv-only", action="store_true", help="print only the conv times (A/B of conv settings)")
    a = ap.parse_args()
    C = native()
    dev = "cuda"
    for H, Cin, Cout in SHAPES:
        N = a.batch
        M, K = N * H * H, 9 * Cin
        A = torch.rand(M, K, device=dev).sub_(0.5).to(torch.bfloat16)
        B = torch.rand(K, Cout, device=dev).sub_(0.5).to(torch.bfloat16)
        x = torch.rand(N, H, H, Cin, device=dev).sub_(0.5).to(torch.bfloat16)
        w = (torch.rand(Cout, K, device=dev).sub_(0.5) * 0.05).to(torch.bfloat16)
        y = torch.empty(N, H, H, Cout, dtype=torch.bfloat16, device=dev)
        stats = torch.zeros(max(C.conv_stats_rows(M, Cout, 0), 1024) * 2 * Cout, device=dev)
        gemm = lambda: torch.matmul(A, B)  # noqa: E731
        conv = lambda: C.conv_fwd(x, None, w, 9, 0, y, None, stats, 0, None, 0)  # noqa: E731
        gemm(), conv()
        torch.cuda.synchronize()
        tg, tc = [], []
        for _ in range(a.rounds):
            tg.append(timed(gemm, a.reps) if not a.conv_only else 1.0)
            tc.append(timed(conv, a.reps))
        if a.conv_only:
            print(f"{N}x{H}x{H} {Cin}->{Cout}: conv {statistics.median(tc) * 1e3:.1f} us", flush=True)
            continue
        flops = 2.0 * M * Cout * K
        g, c = statistics.median(tg), statistics.median(tc)
        print(json.dumps({"shape": f"{N}x{H}x{H} {Cin}->{Cout}", "M": M, "N": Cout, "K": K,
                          "hipblaslt_us": round(g * 1e3, 1), "hipblaslt_tflops": round(flops / g / 1e9, 1),
                          "conv_us": round(c * 1e3, 1), "conv_tflops": round(flops / c / 1e9, 1),
                          "conv_vs_gemm": round(g / c, 3)}), flush=True)


if __name__ == "__main__":
    main()

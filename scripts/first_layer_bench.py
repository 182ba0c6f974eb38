#!/usr/bin/env python3
"""Time the first-layer conv (3 -> 64, packed K) at the training shape: packed implicit GEMM
(bm_pref 256) vs conv_first.hip (bm_pref 13), interleaved rounds, median us."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robotic_discovery_platform_amd.ops import native  # noqa: E402

C = native()
dev = "cuda"
for N in (64, 4, 1):
    H = W = 256
    x8 = torch.zeros(N, H, W, 8, dtype=torch.bfloat16, device=dev)
    x8[..., :3] = torch.rand(N, H, W, 3, device=dev).to(torch.bfloat16)
    wk = (torch.randn(64, 128, device=dev) * 0.1).to(torch.bfloat16)
    y = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=dev)
    rows = C.conv_stats_rows(N * H * W, 64, 0)
    st = torch.zeros(rows * 2 * 64, device=dev)
    times = {256: [], 13: []}
    for p in times:
        C.conv_fwd(x8, None, wk, 9, 1, y, None, st, p, None, 0)
    torch.cuda.synchronize()
    for _ in range(5):
        for p in times:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                C.conv_fwd(x8, None, wk, 9, 1, y, None, st, p, None, 0)
            e1.record()
            torch.cuda.synchronize()
            times[p].append(e0.elapsed_time(e1) / 10 * 1e3)
    print(f"N={N}: packed igemm {statistics.median(times[256]):.1f} us, conv_first {statistics.median(times[13]):.1f} us "
          f"(output {N * H * W * 128 / 1e6:.0f} MB)", flush=True)

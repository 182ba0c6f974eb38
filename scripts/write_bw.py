#!/usr/bin/env python3
"""HBM write / copy bandwidth reference: torch fill_ and copy_ of a 537 MB bf16 tensor (the size of one
256^2 x 64-channel activation at bs 64), median of 10 timed reps."""
import statistics
import torch

n = 64 * 256 * 256 * 64
a = torch.empty(n, dtype=torch.bfloat16, device="cuda")
b = torch.ones(n, dtype=torch.bfloat16, device="cuda")
for name, fn, nbytes in (("fill (write only)", lambda: a.fill_(1.0), 2 * n), ("copy (read + write)", lambda: a.copy_(b), 4 * n)):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    t = statistics.median(ts)
    print(f"{name}: {t:.1f} us, {nbytes / t / 1e6:.2f} TB/s", flush=True)

#!/usr/bin/env python3
"""Is the native training step host-bound? Times the host enqueue of K steps (no sync inside)
against the device time of the same K steps, at the given batch sizes. JSON lines to stdout."""
import json
import sys
import time

import torch


def main():
    sys.path.insert(0, ".")
    from robotic_discovery_platform_amd.train.engine import build_bench_step
    dev = torch.device("cuda")
    for b in [int(x) for x in (sys.argv[1:] or ["4", "64"])]:
        fn = build_bench_step(batch=b, size=256, decoder="bilinear", device=dev, world=1, graph="auto",
                              bucket_mb=16.0)
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        K = 40
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        for _ in range(K):
            fn()
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(json.dumps({"batch": b, "host_enqueue_ms_per_step": round((t1 - t0) * 1e3 / K, 3),
                          "wall_ms_per_step": round((t2 - t0) * 1e3 / K, 3),
                          "device_ms_per_step": round(e0.elapsed_time(e1) / K, 3)}), flush=True)


if __name__ == "__main__":
    main()

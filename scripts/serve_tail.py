#!/usr/bin/env python3
"""Serving tail-latency study: where do the slow frames of the engine and the e2e path come from?

Engine: FramePipeline.process split into submit / wait / host finish per frame (``--frames`` frames,
default 2000), for each variant of (end-event wait: block vs poll ``--spin-us``) x (Python GC: normal vs
``gc.freeze()`` after warm-up). Every frame slower than 2x the median is attributed to the stage that
exceeded its own median by the most, and to a GC pass if one overlapped it (``gc.callbacks``).
E2E: bench_serve.measure_e2e with the same frame count (lock-step p50 / p99 + server stage p99s).

Writes one JSON object to stdout (``profiles/serve_tail.md`` is built from it)."""
import argparse
import gc
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class GcClock:
    def __init__(self):
        self.spans = []
        self._t = None
        gc.callbacks.append(self._cb)

    def _cb(self, phase, info):
        if phase == "start":
            self._t = time.perf_counter()
        elif self._t is not None:
            self.spans.append((self._t, time.perf_counter(), info.get("generation", -1)))
            self._t = None

    def overlaps(self, a, b):
        return [g for (s, e, g) in self.spans if s < b and e > a]


def engine_variant(pipe, scenes, frames, warmup, spin_us, freeze, clock):
    pipe.runner.set_spin_us(spin_us)
    gc.unfreeze()
    gc.collect()
    for i in range(warmup):
        sc = scenes[i % len(scenes)]
        pipe.process(sc.color, sc.depth)
    if freeze:
        gc.freeze()
    clock.spans.clear()
    rows = []
    for i in range(frames):
        sc = scenes[i % len(scenes)]
        t0 = time.perf_counter()
        pipe.submit(sc.color, sc.depth)
        t1 = time.perf_counter()
        r = pipe.collect()
        t2 = time.perf_counter()
        rows.append((t0, t1, t2, r.timings["wait_ms"], r.timings["gpu_ms"]))
    gc.unfreeze()
    tot = np.array([(r[2] - r[0]) * 1e3 for r in rows])
    sub = np.array([(r[1] - r[0]) * 1e3 for r in rows])
    wait = np.array([r[3] for r in rows])
    gpu = np.array([r[4] for r in rows])
    fin = tot - sub - wait
    med = {k: float(np.median(v)) for k, v in (("submit", sub), ("wait", wait), ("finish", fin), ("gpu", gpu))}
    p50 = float(np.median(tot))
    slow = np.nonzero(tot > 2 * p50)[0]
    cause = {}
    for i in slow:
        ex = {"submit": sub[i] - med["submit"], "wait": wait[i] - med["wait"], "finish": fin[i] - med["finish"]}
        k = max(ex, key=ex.get)
        if k == "wait" and gpu[i] > 1.5 * med["gpu"]:
            k = "wait(gpu)"
        if clock.overlaps(rows[i][0], rows[i][2]):
            k += "+gc"
        cause[k] = cause.get(k, 0) + 1
    pct = lambda v, q: round(float(np.percentile(v, q)), 3)  # noqa: E731
    return {"spin_us": spin_us, "gc_freeze": freeze, "frames": frames, "fps": round(1e3 * frames / tot.sum(), 1),
            "p50_ms": pct(tot, 50), "p99_ms": pct(tot, 99), "p999_ms": pct(tot, 99.9), "max_ms": round(float(tot.max()), 3),
            "submit_p50": pct(sub, 50), "submit_p99": pct(sub, 99), "wait_p50": pct(wait, 50), "wait_p99": pct(wait, 99),
            "finish_p50": pct(fin, 50), "finish_p99": pct(fin, 99), "gpu_p50": pct(gpu, 50), "gpu_p99": pct(gpu, 99),
            "slow_frames": int(len(slow)), "slow_causes": cause, "gc_passes": len(clock.spans)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--spin-us", type=float, default=1000.0)
    ap.add_argument("--e2e", type=int, default=1)
    a = ap.parse_args()
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K
    from robotic_discovery_platform_amd.serve.bench_serve import measure_e2e, prepare_model
    from robotic_discovery_platform_amd.serve.engine import FramePipeline
    dev = torch.device("cuda")
    model, scenes = prepare_model(dev, 50)
    pipe = FramePipeline(model, DEFAULT_K, 0.001, graph=True)
    clock = GcClock()
    out = {"engine": []}
    for spin in (0.0, a.spin_us):
        for freeze in (False, True):
            v = engine_variant(pipe, scenes, a.frames, a.warmup, spin, freeze, clock)
            print(f"[tail] {v}", file=sys.stderr, flush=True)
            out["engine"].append(v)
    if a.e2e:
        out["e2e"] = measure_e2e(model, scenes, a.frames, a.warmup)
    print(json.dumps(out), flush=True)
    sys.stdout.flush()
    os._exit(0)  # (gRPC core threads at interpreter exit)


if __name__ == "__main__":
    main()

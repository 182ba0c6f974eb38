"""Host-side cost of one engine frame (submit_color / submit_depth / collect), native FrameRunner path vs
the Python (torch) path of the same FramePipeline, one MI355X. JSON lines."""
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K  # noqa: E402
from robotic_discovery_platform_amd.serve.engine import FramePipeline  # noqa: E402

from robotic_discovery_platform_amd.serve.bench_serve import prepare_model  # noqa: E402
m, scenes = prepare_model(torch.device("cuda"), 200)  # trained briefly: realistic masks / edge counts
p = FramePipeline(m, DEFAULT_K, 0.001, graph=True)
sc = scenes[1]
runner = p.runner
for name, r in (("native", runner), ("python", None), ("native2", runner)):
    p.runner = r
    t = {"color": [], "depth": [], "wait": [], "collect": [], "total": []}
    for i in range(300):
        t0 = time.perf_counter()
        p.submit_color(sc.color)
        t1 = time.perf_counter()
        p.submit_depth(sc.depth)
        t2 = time.perf_counter()
        torch.cuda.current_stream()  # no-op
        res = p.collect()
        t3 = time.perf_counter()
        if i >= 50:
            t["color"].append((t1 - t0) * 1e3)
            t["depth"].append((t2 - t1) * 1e3)
            t["wait"].append(res.timings["wait_ms"])
            t["collect"].append((t3 - t2) * 1e3)
            t["total"].append((t3 - t0) * 1e3)
    print(json.dumps({"path": name, **{k: round(statistics.median(v), 4) for k, v in t.items()},
                      "gpu_ms": round(res.timings["gpu_ms"], 4)}), flush=True)

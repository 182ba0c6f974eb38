"""Serving e2e A/B on one GPU: the gRPC service with its per-stage breakdown under several server
settings (GIL switch interval; client streams; server processes). One JSON line per configuration.

    python scripts/serve_e2e_ab.py [--frames 300] [--switch 0,0.5,0.1] [--streams 1,4]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from robotic_discovery_platform_amd.serve.bench_serve import measure_e2e, measure_e2e_procs, prepare_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=300)
ap.add_argument("--warmup", type=int, default=30)
ap.add_argument("--switch", default="0,0.5,0.1")
ap.add_argument("--streams", default="1,4")
ap.add_argument("--null", type=int, default=0, help="host path only (NullEngine)")
ap.add_argument("--procs", default="", help="server-process configs procs:streams[:hw_queues],... (measure_e2e_procs)")
a = ap.parse_args()
model = None
if not a.null:
    model, _ = prepare_model(torch.device("cuda"), 200)
for sw in (float(x) for x in a.switch.split(",")):
    for st in (int(x) for x in a.streams.split(",")):
        r = measure_e2e(model, None, a.frames, a.warmup, streams=st, switch_ms=sw)
        print(json.dumps({"switch_ms": sw, "streams": st, "null_engine": bool(a.null), **r}), flush=True)
for spec in filter(None, a.procs.split(",")):
    pr, st, *hq = (int(x) for x in spec.split(":"))
    r = measure_e2e_procs(model, a.frames, a.warmup, procs=pr, streams=st, hw_queues=hq[0] if hq else 0)
    print(json.dumps({"procs": pr, "streams": st, **r}), flush=True)

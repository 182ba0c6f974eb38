#!/usr/bin/env python3
"""Host decode times of one served request (the colour JPEG's entropy decode and the depth PNG's inflate),
serial and on the shared host pool (RDP_HOST_THREADS), median of 300. usage: host_decode_bench.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robotic_discovery_platform_amd.data.image_io import decode_image  # noqa: E402
from robotic_discovery_platform_amd.data.jpeg import decode_coefs  # noqa: E402
from robotic_discovery_platform_amd.data.synthetic import make_scene  # noqa: E402
from robotic_discovery_platform_amd.serve.client import make_request  # noqa: E402


def med(fn, n=300):
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return round(float(np.median(ts)) * 1e3, 4)


sc = make_scene(3)
rq = make_request(sc.color, sc.depth)
jb, pb = rq.color_image.data, rq.depth_image.data
out = {"threads": os.environ.get("RDP_HOST_THREADS", "default"), "jpeg_bytes": len(jb), "png_bytes": len(pb),
       "jpeg_serial_ms": med(lambda: decode_coefs(jb, parallel=False, pin=False)),
       "jpeg_parallel_ms": med(lambda: decode_coefs(jb, parallel=True, pin=False)),
       "png_ms": med(lambda: decode_image(pb, False))}
print(json.dumps(out), flush=True)

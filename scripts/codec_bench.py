"""Host codec timings of one serving frame (640x480): colour JPEG (PIL decode vs native entropy
decode, serial / restart-parallel) and depth PNG (PIL vs native, plain / banded-parallel), alone and
with several caller threads (the server's codec pool). Prints one JSON line.

    python scripts/codec_bench.py [--iters 200] [--threads 1,4,8]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from robotic_discovery_platform_amd.data.image_io import decode_image, encode_jpeg, encode_png  # noqa: E402
from robotic_discovery_platform_amd.data.jpeg import decode_coefs  # noqa: E402
from robotic_discovery_platform_amd.data.synthetic import make_scene  # noqa: E402
from robotic_discovery_platform_amd.ops import native  # noqa: E402


def timed(fn, iters, threads):
    """median per-call ms with `threads` concurrent callers"""
    lat = [[] for _ in range(threads)]

    def run(k):
        for _ in range(iters):
            t = time.perf_counter()
            fn()
            lat[k].append((time.perf_counter() - t) * 1e3)
    fn()
    th = [threading.Thread(target=run, args=(k,)) for k in range(threads)]
    t0 = time.perf_counter()
    [t.start() for t in th]
    [t.join() for t in th]
    wall = time.perf_counter() - t0
    allv = np.concatenate([np.asarray(v) for v in lat])
    return {"p50_ms": round(float(np.median(allv)), 3), "calls_per_s": round(threads * iters / wall, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--threads", default="1,4,8")
    a = ap.parse_args()
    C = native(build_if_missing=False)
    assert C is not None, "native extension missing"
    sc = make_scene(3)
    jpg_plain = encode_jpeg(sc.color, 95)
    jpg_rst = encode_jpeg(sc.color, 95, restart_rows=1)
    png_plain = encode_png(sc.depth, 1)
    png_band = encode_png(sc.depth, 1, bands=8)
    cases = {
        "jpeg_pil": lambda: decode_image(jpg_rst, True, "RGB"),
        "jpeg_native_serial": lambda: decode_coefs(jpg_rst, parallel=False),
        "jpeg_native_parallel": lambda: decode_coefs(jpg_rst, parallel=True),
        "jpeg_native_norestart": lambda: decode_coefs(jpg_plain, parallel=True),
        "png_native_plain": lambda: C.png_decode(png_plain, True),
        "png_native_banded_serial": lambda: C.png_decode(png_band, False),
        "png_native_banded_parallel": lambda: C.png_decode(png_band, True),
        "png_encode_mask_1band": lambda: encode_png(sc.mask, 1, bands=1),
        "png_encode_mask_4bands": lambda: encode_png(sc.mask, 1, bands=4),
    }
    out = {"frame": "640x480", "jpeg_bytes": len(jpg_rst), "png_bytes": len(png_band), "cpus": os.cpu_count()}
    for th in (int(x) for x in a.threads.split(",")):
        for k, fn in cases.items():
            out[f"{k}_t{th}"] = timed(fn, a.iters if th == 1 else max(20, a.iters // 2), th)
            print(f"[codec_bench] {k} threads={th} {out[f'{k}_t{th}']}", file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

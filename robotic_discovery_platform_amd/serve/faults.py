"""Fault injection for the serving path (tests and chaos runs).

The reference has no fault injection (SURVEY.md §5 "Failure detection"); its failure semantics are
"any per-frame exception -> StatusCode.INTERNAL + one empty response" (``/root/reference/services/
vision_analysis/server.py:154-158``) and "degenerate geometry -> all-zero CurvatureResult"
(``/root/reference/pkg/geometry_utils.py:64-70,95-97``). ``FaultInjector`` corrupts chosen requests
before they are decoded so those paths can be exercised deterministically:

  * ``truncated_png``  depth PNG cut to half its bytes        -> decode error -> degraded response
  * ``corrupt_jpeg``   colour JPEG bytes scrambled after the header -> decode error or garbage frame
  * ``zero_depth``     depth replaced by an all-zero 16-bit PNG -> no valid points -> too_few_points
  * ``size_mismatch``  depth re-encoded at half resolution     -> engine shape error -> degraded
  * ``empty_color``    colour payload emptied                   -> decode error -> degraded

Configure programmatically (``FaultInjector({"truncated_png": [3, 7]})``: frame indices per stream)
or from ``RDP_FAULT_INJECT="truncated_png@3,7;zero_depth@5"`` via :func:`from_env`.
"""
from __future__ import annotations

import io
import os
import threading
from typing import Dict, Iterable, Optional, Tuple

import numpy as np

KINDS = ("truncated_png", "corrupt_jpeg", "zero_depth", "size_mismatch", "empty_color")


class FaultInjector:
    def __init__(self, plan: Dict[str, Iterable[int]]):
        bad = set(plan) - set(KINDS)
        if bad:
            raise ValueError(f"unknown fault kinds {sorted(bad)}; known: {KINDS}")
        self.by_frame: Dict[int, str] = {}
        for kind, frames in plan.items():
            for f in frames:
                self.by_frame[int(f)] = kind
        self.injected: Dict[str, int] = {k: 0 for k in KINDS}
        self._lock = threading.Lock()

    def corrupt_request(self, index: int, color: bytes, depth: bytes) -> Tuple[bytes, bytes]:
        kind = self.by_frame.get(index)
        if kind is None:
            return color, depth
        with self._lock:
            self.injected[kind] += 1
        if kind == "truncated_png":
            return color, depth[: max(1, len(depth) // 2)]
        if kind == "corrupt_jpeg":
            rng = np.random.default_rng(index)
            b = bytearray(color)
            lo = min(len(b), 600)  # keep the SOI/APP headers, scramble the entropy-coded data
            if len(b) > lo:
                b[lo:] = rng.integers(0, 256, len(b) - lo, dtype=np.uint8).tobytes()
            return bytes(b), depth
        if kind == "empty_color":
            return b"", depth
        if kind in ("zero_depth", "size_mismatch"):
            from ..data.image_io import decode_image, encode_png
            d = decode_image(depth, False)
            if kind == "zero_depth":
                d = np.zeros_like(d)
            else:
                d = np.ascontiguousarray(d[::2, ::2])
            return color, encode_png(d)
        return color, depth


def from_env(var: str = "RDP_FAULT_INJECT") -> Optional[FaultInjector]:
    spec = os.environ.get(var, "").strip()
    if not spec:
        return None
    plan: Dict[str, list] = {}
    for part in spec.split(";"):
        kind, _, frames = part.partition("@")
        plan.setdefault(kind.strip(), []).extend(int(f) for f in frames.split(",") if f.strip())
    return FaultInjector(plan)

"""ROCTx ranges around pipeline stages (SURVEY.md §5 "Tracing / profiling").

``with trace.range("fwd"):`` pushes a roctx range visible in ``rocprofv3 --marker-trace`` /
Perfetto timelines when ``RDP_ROCTX=1``; otherwise it costs one dict lookup. The library is
loaded with ctypes (``libroctx64.so`` ships with ROCm) so no extension rebuild is needed; inside a
hipGraph capture the markers record host-side phases only (graph replays are one launch).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Optional

_lib: Optional[ctypes.CDLL] = None
_enabled = os.environ.get("RDP_ROCTX", "0") == "1"


def _load() -> Optional[ctypes.CDLL]:
    global _lib, _enabled
    if _lib is None and _enabled:
        for name in ("libroctx64.so", "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"):
            try:
                _lib = ctypes.CDLL(name)
                _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                break
            except OSError:
                continue
        if _lib is None:
            _enabled = False
    return _lib


def enable(on: bool = True) -> bool:
    """Turn markers on/off at runtime; returns whether the roctx library is usable."""
    global _enabled
    _enabled = on
    return _load() is not None if on else False


def enabled() -> bool:
    return _enabled and _load() is not None


_NULL = contextlib.nullcontext()


def range(name: str):  # noqa: A001 - mirrors roctxRange naming
    """A roctx range context; markers off: one shared no-op context (no generator per call -- several
    ranges sit on every served frame's path)."""
    lib = _load() if _enabled else None
    if lib is None:
        return _NULL
    return _roctx_range(lib, name)


@contextlib.contextmanager
def _roctx_range(lib, name: str):
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _load() if _enabled else None
    if lib is not None:
        lib.roctxMarkA(name.encode())

"""Native HIP/CDNA4 op library (``robotic_discovery_platform_amd/_C.so``).

``native()`` returns the compiled extension. On a GPU box it MUST be present: there is no silent
eager fallback for GPU tensors -- the plain-torch model (:mod:`..models.unet_ref`) and the numpy /
scipy geometry (:mod:`..geometry.reference`) are test oracles and the CPU path only.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None


def native(build_if_missing: bool = True):
    """Import (building in-tree first if needed) the native kernel library."""
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        import torch  # noqa: F401  (loads libtorch before the extension)
        alt = os.environ.get("RDP_NATIVE_SO")  # A/B runs: load another build of the same library
        if alt:
            from importlib import machinery, util
            loader = machinery.ExtensionFileLoader("robotic_discovery_platform_amd._C", alt)
            spec = util.spec_from_file_location("robotic_discovery_platform_amd._C", alt, loader=loader)
            _mod = util.module_from_spec(spec)
            loader.exec_module(_mod)
            return _mod
        try:
            _mod = importlib.import_module("robotic_discovery_platform_amd._C")
        except ImportError as e:
            if not build_if_missing or os.environ.get("RDP_NO_BUILD"):
                raise RuntimeError(
                    "robotic_discovery_platform_amd._C is not built; run "
                    "`python -m robotic_discovery_platform_amd._build`") from e
            from .. import _build
            _build.build(verbose=True)
            _mod = importlib.import_module("robotic_discovery_platform_amd._C")
    return _mod


def available() -> bool:
    try:
        native(build_if_missing=False)
        return True
    except Exception:
        return False

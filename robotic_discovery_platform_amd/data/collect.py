"""Raw RGB-D collection + labelling into the training layout.

Collection = ``/root/reference/scripts/02_collect_segmentation_data.py:40-117``: frames from the
camera are written every ``save_interval_s`` (0.5 s) to ``ml/raw_data/capture_<unix>/`` as
``color/color_<ts>.png`` (BGR PNG) and ``depth/depth_<ts>.npy`` (raw uint16), with ``<ts>`` =
``f"{time.time():.2f}"`` with the dot replaced by ``_``. The reference toggles saving with a key and
shows an overlay; headless here, collection runs for ``n_frames`` or ``duration_s``.

The reference README promises "collect and auto-label" but ships no labeller;
``label_capture`` turns a capture into ``ml/datasets/processed/{images,masks}`` (identical file
names, the pairing ``SegmentationDataset`` expects) using the depth auto-labeller.
"""
from __future__ import annotations

import glob
import logging
import os
import time
from typing import Callable, Optional, Tuple

import numpy as np

from ..config import CollectConfig
from .image_io import imread, imwrite
from .synthetic import auto_label

log = logging.getLogger(__name__)


def collect_raw_data(cam, cfg: Optional[CollectConfig] = None, n_frames: Optional[int] = None,
                     duration_s: Optional[float] = None, out_dir: Optional[str] = None) -> Tuple[str, int]:
    cfg = cfg or CollectConfig()
    out_dir = out_dir or os.path.join(cfg.raw_dir, f"capture_{int(time.time())}")
    cdir, ddir = os.path.join(out_dir, "color"), os.path.join(out_dir, "depth")
    os.makedirs(cdir, exist_ok=True)
    os.makedirs(ddir, exist_ok=True)
    saved, last_save, t_start = 0, 0.0, time.time()
    last_frame = -1
    while (n_frames is None or saved < n_frames) and (duration_s is None or time.time() - t_start < duration_s):
        if getattr(cam, "frame_count", None) == last_frame:
            time.sleep(0.001)
            continue
        depth_frame, color = cam.get_frames()
        if color is None or depth_frame is None:
            time.sleep(0.001)
            continue
        last_frame = getattr(cam, "frame_count", None)
        now = time.time()
        if now - last_save < cfg.save_interval_s:
            continue
        ts = f"{now:.2f}".replace(".", "_")
        if os.path.exists(os.path.join(cdir, f"color_{ts}.png")):
            ts = f"{ts}_{saved}"
        imwrite(os.path.join(cdir, f"color_{ts}.png"), color)
        np.save(os.path.join(ddir, f"depth_{ts}.npy"), np.asanyarray(depth_frame.get_data()))
        saved += 1
        last_save = now
    log.info("saved %d frame pairs to %s", saved, out_dir)
    return out_dir, saved


def label_capture(capture_dir: str, processed_dir: str, depth_scale: float = 0.001,
                  labeler: Optional[Callable[[np.ndarray, np.ndarray], np.ndarray]] = None) -> int:
    """Write images/ + masks/ pairs (same file name) from a capture directory."""
    img_dir, mask_dir = os.path.join(processed_dir, "images"), os.path.join(processed_dir, "masks")
    os.makedirs(img_dir, exist_ok=True)
    os.makedirs(mask_dir, exist_ok=True)
    n = 0
    for cpath in sorted(glob.glob(os.path.join(capture_dir, "color", "color_*.png"))):
        ts = os.path.basename(cpath)[len("color_"):-len(".png")]
        dpath = os.path.join(capture_dir, "depth", f"depth_{ts}.npy")
        if not os.path.exists(dpath):
            continue
        color = imread(cpath)
        depth = np.load(dpath, allow_pickle=False)
        mask = labeler(color, depth) if labeler else auto_label(depth, depth_scale)
        name = f"{os.path.basename(os.path.normpath(capture_dir))}_{ts}.png"
        imwrite(os.path.join(img_dir, name), color)
        imwrite(os.path.join(mask_dir, name), mask)
        n += 1
    return n

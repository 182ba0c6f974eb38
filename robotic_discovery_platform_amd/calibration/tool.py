"""Calibration workflow (headless version of ``/root/reference/scripts/01_calibrate_camera.py``).

The reference loop shows the live stream, captures a view on ``c`` (corners found + refined),
finishes on ``q`` once >= 5 views exist, runs ``calibrateCamera``, saves ``mtx, dist, rvecs, tvecs``
with ``np.savez`` and prints the mean reprojection error (``:60-112``). Here the same steps run
over frames from any camera source (``capture`` views) or over image files, and the result goes
to ``CalibrationConfig.out_file`` = ``ml/configs/calibration_data.npz`` -- the path the server and
client read (the reference writes ``ml/data/``) -- including the camera's
``depth_scale`` when it reports one.
"""
from __future__ import annotations

import glob
import logging
import threading
from typing import Iterable, List, Optional, Tuple

import numpy as np

from ..camera import BaseCamera, DepthFrame, write_calibration
from ..config import CalibrationConfig
from .board import object_points, random_board_pose, render_board_view
from .corners import corner_subpix, find_chessboard_corners
from .zhang import calibrate_camera, reprojection_errors

log = logging.getLogger(__name__)


class SyntheticBoardCamera(BaseCamera):
    """Shows a checkerboard at random poses through a known lens (ground truth for the tool)."""

    def __init__(self, width=640, height=480, fps=30, K=None, dist=None, pattern=(9, 7), square=0.027, seed=0,
                 depth_scale: float = 0.001, ss: int = 2):
        super().__init__(width, height, fps)
        self.K = np.array([[615.0, 0, width / 2 + 2.5], [0, 612.0, height / 2 - 2.0], [0, 0, 1]]) if K is None else K
        self.dist = np.array([0.06, -0.12, 0.0008, -0.0004, 0.02]) if dist is None else dist
        self.pattern, self.square, self.ss = pattern, square, ss
        self.rng = np.random.default_rng(seed)
        self._scale = depth_scale
        self._i = 0

    def _open(self):
        self.depth_scale = self._scale

    def _grab(self):
        r, t = random_board_pose(self.rng, self.K, self.pattern, self.square, (self.width, self.height), self.dist)
        g = render_board_view(self.K, self.dist, r, t, self.pattern, self.square, (self.width, self.height),
                              ss=self.ss, seed=self._i)
        self._i += 1
        color = np.repeat(g[..., None], 3, -1)
        depth = np.full((self.height, self.width), int(round(float(t[2]) / self._scale)), np.uint16)
        self.stopped.wait(1.0 / self.fps)
        return DepthFrame(depth, self._scale), color


def detect_view(img: np.ndarray, cfg: CalibrationConfig) -> Optional[np.ndarray]:
    gray = img if img.ndim == 2 else img[..., :3].mean(-1)
    ok, c = find_chessboard_corners(gray, tuple(cfg.checkerboard))
    if not ok:
        return None
    return corner_subpix(gray, c, tuple(cfg.subpix_window), cfg.subpix_max_iter, cfg.subpix_eps)


def calibrate_views(images: Iterable[np.ndarray], cfg: Optional[CalibrationConfig] = None):
    """Detect + calibrate; returns dict(rms, mtx, dist, rvecs, tvecs, mean_error, n_views, size)."""
    cfg = cfg or CalibrationConfig()
    objp = object_points(tuple(cfg.checkerboard), cfg.square_size_m)
    objs: List[np.ndarray] = []
    imgs: List[np.ndarray] = []
    size = None
    for img in images:
        size = (img.shape[1], img.shape[0])
        c = detect_view(img, cfg)
        if c is None:
            log.info("checkerboard not found in a view; skipped")
            continue
        objs.append(objp)
        imgs.append(c)
    if len(objs) < cfg.min_captures:
        raise RuntimeError(f"need at least {cfg.min_captures} views with a detected board, got {len(objs)}")
    rms, mtx, dist, rvecs, tvecs = calibrate_camera(objs, imgs, size)
    errs = reprojection_errors(objs, imgs, mtx, dist, rvecs, tvecs)
    return dict(rms=rms, mtx=mtx, dist=dist, rvecs=rvecs, tvecs=tvecs, mean_error=float(np.mean(errs)),
                n_views=len(objs), size=size)


def run_calibration(cfg: Optional[CalibrationConfig] = None, cam: Optional[BaseCamera] = None,
                    image_glob: Optional[str] = None, n_captures: int = 10, out_file: Optional[str] = None) -> dict:
    """Capture (or read) views, calibrate, save the npz; returns the calibration dict."""
    from ..data.image_io import imread
    cfg = cfg or CalibrationConfig()
    depth_scale = None
    if image_glob:
        views = [imread(p) for p in sorted(glob.glob(image_glob))]
    else:
        own = cam is None
        cam = cam or SyntheticBoardCamera()
        if own and not cam.start():
            raise RuntimeError("failed to start camera")
        views = []
        last = -1
        try:
            while len(views) < n_captures:
                if cam.frame_count == last:
                    threading.Event().wait(0.001)
                    continue
                last = cam.frame_count
                _, color = cam.get_frames()
                if color is not None:
                    views.append(color)
            depth_scale = cam.get_depth_scale()
        finally:
            if own:
                cam.stop()
    res = calibrate_views(views, cfg)
    path = out_file or cfg.out_file
    write_calibration(path, res["mtx"], res["dist"], np.stack(res["rvecs"]), np.stack(res["tvecs"]), depth_scale)
    res["path"] = path
    log.info("calibration saved to %s (rms %.4f px, mean reprojection error %.4f px over %d views)", path,
             res["rms"], res["mean_error"], res["n_views"])
    return res

"""RGB-D camera sources with the reference ``Camera`` interface.

Interface = ``/root/reference/pkg/camera.py:29-161``: ``Camera(width=640, height=480, fps=30)``,
``start() -> bool``, ``stop()``, a daemon background thread keeping only the latest frame under a
lock (latest-frame-wins, ``:89-115``), non-blocking ``get_frames() -> (depth_frame, color_copy)``
returning ``(None, None)`` before the first frame (``:117-134``), ``load_intrinsics(path) ->
(mtx, dist)`` (``:136-155``) and ``get_depth_scale()`` (``:157-161``).

Backends:
  * ``SyntheticCamera`` (default here: no camera or librealsense in this environment) renders the
    bending-actuator scenes of ``data/synthetic.py`` at ``fps``; its depth frames behave like
    ``rs.depth_frame`` (``get_data()``, ``get_width()``, ``get_height()``, ``get_distance()``).
  * ``RealSenseCamera`` wraps pyrealsense2 (z16 + bgr8, depth aligned to colour) when importable.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from typing import Optional, Tuple

import numpy as np

log = logging.getLogger(__name__)


class DepthFrame:
    """Array-backed stand-in for ``rs.depth_frame`` (z16 in ``depth_scale`` units)."""

    def __init__(self, data: np.ndarray, depth_scale: float):
        self._d = data
        self._s = depth_scale

    def get_data(self) -> np.ndarray:
        return self._d

    def get_width(self) -> int:
        return int(self._d.shape[1])

    def get_height(self) -> int:
        return int(self._d.shape[0])

    def get_distance(self, x: int, y: int) -> float:
        return float(self._d[y, x]) * self._s

    def __bool__(self) -> bool:
        return True


class BaseCamera:
    def __init__(self, width: int = 640, height: int = 480, fps: int = 30):
        self.width, self.height, self.fps = width, height, fps
        self.depth_scale: Optional[float] = None
        self.frame_lock = threading.Lock()
        self.stopped = threading.Event()
        self.latest_frame = None
        self.frame_count = 0
        self.thread = threading.Thread(target=self._read_loop, daemon=True)

    # -- to implement
    def _open(self) -> None:
        raise NotImplementedError

    def _grab(self):
        """Block until the next frame; return (depth_frame, color_bgr) or None."""
        raise NotImplementedError

    def _close(self) -> None:
        pass

    # -- reference surface
    def start(self) -> bool:
        try:
            self._open()
            self.thread.start()
            log.info("camera started (%s %dx%d@%d)", type(self).__name__, self.width, self.height, self.fps)
            return True
        except Exception as e:  # reference: log + False (camera.py:77-79)
            log.error("failed to start camera: %s", e)
            return False

    def stop(self) -> None:
        self.stopped.set()
        if self.thread.is_alive():
            self.thread.join()
        self._close()

    def _read_loop(self) -> None:
        while not self.stopped.is_set():
            try:
                fr = self._grab()
                if fr is None:
                    continue
                with self.frame_lock:
                    self.latest_frame = fr
                    self.frame_count += 1
            except RuntimeError as e:  # reference: warn + back off (camera.py:112-115)
                log.warning("frame reading error in background thread: %s", e)
                time.sleep(0.1)

    def get_frames(self):
        with self.frame_lock:
            if self.latest_frame is None:
                return None, None
            depth_frame, color = self.latest_frame
            return depth_frame, color.copy()

    def wait_for_first_frame(self, timeout: float = 5.0) -> bool:
        t0 = time.time()
        while time.time() - t0 < timeout:
            with self.frame_lock:
                if self.latest_frame is not None:
                    return True
            time.sleep(0.001)
        return False

    @staticmethod
    def load_intrinsics(calib_path: str) -> Tuple[Optional[np.ndarray], Optional[np.ndarray]]:
        if not os.path.exists(calib_path):
            log.error("calibration file not found at '%s' (run the calibration script first)", calib_path)
            return None, None
        with np.load(calib_path, allow_pickle=False) as data:
            return data["mtx"], data["dist"]

    def get_depth_scale(self) -> Optional[float]:
        if self.depth_scale is None:
            log.warning("depth scale not available; is the camera started?")
        return self.depth_scale


class SyntheticCamera(BaseCamera):
    """Renders a bending actuator whose radius sweeps over time (a known curvature signal)."""

    def __init__(self, width: int = 640, height: int = 480, fps: int = 30, n_scenes: int = 16, seed: int = 0,
                 depth_scale: float = 0.001, realtime: bool = True):
        super().__init__(width, height, fps)
        self._n, self._seed, self._scale, self._rt = n_scenes, seed, depth_scale, realtime
        self._scenes = []
        self._i = 0
        self._t_next = 0.0

    def _open(self) -> None:
        from ..data.synthetic import DEFAULT_K, make_scene
        K = DEFAULT_K.copy()
        K[0, 2], K[1, 2] = self.width / 2, self.height / 2
        self.K = K
        radii = np.linspace(0.07, 0.14, self._n)
        self._scenes = [make_scene(self._seed + i, self.width, self.height, K=K, depth_scale=self._scale,
                                   radius_m=float(r)) for i, r in enumerate(radii)]
        self.depth_scale = self._scale
        self._t_next = time.perf_counter()

    def _grab(self):
        if self._rt:
            self._t_next += 1.0 / self.fps
            dt = self._t_next - time.perf_counter()
            if dt > 0:
                time.sleep(dt)
            else:
                self._t_next = time.perf_counter()
        sc = self._scenes[self._i % len(self._scenes)]
        self._i += 1
        return DepthFrame(sc.depth, self._scale), sc.color

    def scene(self, i: int):
        return self._scenes[i % len(self._scenes)]


class RealSenseCamera(BaseCamera):  # pragma: no cover - needs hardware + pyrealsense2
    def _open(self) -> None:
        import pyrealsense2 as rs
        self._rs = rs
        self.pipeline = rs.pipeline()
        cfg = rs.config()
        cfg.enable_stream(rs.stream.depth, self.width, self.height, rs.format.z16, self.fps)
        cfg.enable_stream(rs.stream.color, self.width, self.height, rs.format.bgr8, self.fps)
        self.profile = self.pipeline.start(cfg)
        self.align = rs.align(rs.stream.color)
        self.depth_scale = self.profile.get_device().first_depth_sensor().get_depth_scale()

    def _grab(self):
        frames = self.align.process(self.pipeline.wait_for_frames())
        d, c = frames.get_depth_frame(), frames.get_color_frame()
        if not d or not c:
            return None
        return d, np.asanyarray(c.get_data())

    def _close(self) -> None:
        self.pipeline.stop()


def realsense_available() -> bool:
    try:
        import pyrealsense2  # noqa: F401
        return True
    except Exception:
        return False


def Camera(width: int = 640, height: int = 480, fps: int = 30, backend: str = "auto", **kw) -> BaseCamera:
    """Factory with the reference constructor signature; ``backend`` = auto | synthetic | realsense."""
    if backend == "realsense" or (backend == "auto" and realsense_available()):
        return RealSenseCamera(width, height, fps)
    return SyntheticCamera(width, height, fps, **kw)


def write_calibration(path: str, mtx: np.ndarray, dist: Optional[np.ndarray] = None, rvecs=None, tvecs=None,
                      depth_scale: Optional[float] = None) -> None:
    """npz schema of the reference calibration tool (scripts/01_calibrate_camera.py:104) + optional depth_scale."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    arrs = dict(mtx=np.asarray(mtx, np.float64), dist=np.zeros((1, 5)) if dist is None else np.asarray(dist),
                rvecs=np.zeros((0, 3, 1)) if rvecs is None else np.asarray(rvecs),
                tvecs=np.zeros((0, 3, 1)) if tvecs is None else np.asarray(tvecs))
    if depth_scale is not None:
        arrs["depth_scale"] = np.asarray(depth_scale, np.float64)
    np.savez(path, **arrs)


def load_calibration(path: str, default_depth_scale: float = 0.001):
    """(mtx, dist, depth_scale) — depth_scale optional in the file (server.py:88-98)."""
    with np.load(path, allow_pickle=False) as d:
        ds = float(d["depth_scale"]) if "depth_scale" in d.files else default_depth_scale
        return d["mtx"], (d["dist"] if "dist" in d.files else np.zeros((1, 5))), ds

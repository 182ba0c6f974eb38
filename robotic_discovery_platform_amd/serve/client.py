"""Streaming client / visualiser for VisionAnalysisService.

Behaviour of ``/root/reference/services/vision_analysis/client.py:22-152``: frames from a camera are
JPEG (colour) / 16-bit PNG (depth) encoded into ``AnalysisRequest``s (``:47-74``); the colour frame is
queued (``deque(maxlen=20)``) and paired FIFO with each response (``:92,107``); the mask is
overlaid in red (``addWeighted`` 1.0/0.5, ``:110-116``), the 3-D spline projected with the intrinsics
and distortion (``cv2.projectPoints`` with zero pose, ``:119-125``) and drawn as a green polyline;
curvatures are smoothed over 10 frames (``:128-136``).

No display or OpenCV here, so the visualiser is headless: overlays are composed in numpy and can be
written to ``save_dir``; ``run_client`` returns per-frame records (curvatures, coverage, server
proc time, client round-trip) so it doubles as a load generator. Unlike the reference generator,
which busy-spins and can resend the same latest frame, requests are produced once per new frame.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from collections import deque
from typing import List, Optional

import numpy as np

from ..config import ClientConfig
from ..data.image_io import decode_image, encode_jpeg, encode_png, imwrite
from ..proto import vision as pb

log = logging.getLogger(__name__)


def project_points(pts: np.ndarray, K: np.ndarray, dist: Optional[np.ndarray] = None) -> np.ndarray:
    """cv2.projectPoints(pts, rvec=0, tvec=0, K, dist) for the 5-parameter (k1,k2,p1,p2,k3) model."""
    pts = np.asarray(pts, np.float64).reshape(-1, 3)
    z = pts[:, 2]
    z = np.where(z != 0, z, 1.0)
    x, y = pts[:, 0] / z, pts[:, 1] / z
    d = np.zeros(5) if dist is None else np.asarray(dist, np.float64).ravel()
    d = np.pad(d, (0, max(0, 5 - d.size)))[:5]
    k1, k2, p1, p2, k3 = d
    r2 = x * x + y * y
    radial = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 ** 3
    xd = x * radial + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * radial + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return np.stack([K[0, 0] * xd + K[0, 2], K[1, 1] * yd + K[1, 2]], 1)


def _draw_polyline(img: np.ndarray, pts: np.ndarray, color, thickness: int = 2) -> None:
    H, W = img.shape[:2]
    r = thickness // 2
    for (x0, y0), (x1, y1) in zip(pts[:-1], pts[1:]):
        n = int(max(abs(x1 - x0), abs(y1 - y0))) + 1
        xs = np.rint(np.linspace(x0, x1, n)).astype(int)
        ys = np.rint(np.linspace(y0, y1, n)).astype(int)
        for dy in range(-r, r + 1):
            for dx in range(-r, r + 1):
                xx, yy = xs + dx, ys + dy
                ok = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
                img[yy[ok], xx[ok]] = color


def render_overlay(color_bgr: np.ndarray, resp, K: np.ndarray, dist: Optional[np.ndarray]) -> np.ndarray:
    out = color_bgr.copy()
    if resp.mask:
        m = decode_image(resp.mask, color=False)
        if m is not None and m.shape == out.shape[:2]:
            red = np.zeros_like(out)
            red[m > 0] = (0, 0, 255)
            out = np.clip(out.astype(np.int16) + (red.astype(np.int16) * 0.5).round().astype(np.int16), 0,
                          255).astype(np.uint8)
    if len(resp.spline_points):
        p3 = np.array([(p.x, p.y, p.z) for p in resp.spline_points], np.float32)
        ip = project_points(p3, K, dist).astype(np.int32)
        _draw_polyline(out, ip, (0, 255, 0), 2)
    return out


def make_request(color_bgr: np.ndarray, depth_u16: np.ndarray, jpeg_quality: int = 95, restart_rows: int = 1,
                 png_bands: int = 8):
    """One request: colour as baseline JPEG with a restart marker per MCU row, depth as a 16-bit PNG
    in ``png_bands`` deflate bands -- both standard files any decoder reads, which the server's native
    decoders split across threads (data/jpeg.py, csrc/codecs.cpp)."""
    h, w = color_bgr.shape[:2]
    dh, dw = depth_u16.shape[:2]
    jpg = encode_jpeg(color_bgr, jpeg_quality, restart_rows)
    return pb.AnalysisRequest(color_image=pb.Image(data=jpg, width=w, height=h),
                              depth_image=pb.Image(data=encode_png(depth_u16, compress_level=1, bands=png_bands), width=dw,
                                                   height=dh))


def generate_requests(cam, frame_queue: deque, max_frames: Optional[int] = None,
                      stop: Optional[threading.Event] = None, sent_times: Optional[deque] = None):
    """Yield one request per new camera frame; the colour frame goes to ``frame_queue`` for pairing."""
    last = -1
    n = 0
    while (max_frames is None or n < max_frames) and not (stop is not None and stop.is_set()):
        cnt = getattr(cam, "frame_count", None)
        if cnt is not None and cnt == last:
            time.sleep(0.0005)
            continue
        depth_frame, color = cam.get_frames()
        if color is None or depth_frame is None:
            time.sleep(0.0005)
            continue
        last = cnt
        frame_queue.append(color)
        depth = np.asanyarray(depth_frame.get_data())
        if sent_times is not None:
            sent_times.append(time.perf_counter())
        yield make_request(color, depth)
        n += 1


def run_client(cfg: Optional[ClientConfig] = None, cam=None, max_frames: Optional[int] = None,
               save_dir: Optional[str] = None, render: bool = False) -> List[dict]:
    import grpc
    from ..camera import Camera
    cfg = cfg or ClientConfig()
    own_cam = cam is None
    if cam is None:
        cam = Camera()
        if not cam.start():
            log.error("failed to start camera")
            return []
    K, dist = cam.load_intrinsics(cfg.calib_file)
    if K is None:
        K = getattr(cam, "K", None)
        if K is None:
            log.error("could not load camera calibration from %s", cfg.calib_file)
            if own_cam:
                cam.stop()
            return []
        dist = np.zeros((1, 5))
    frame_queue: deque = deque(maxlen=cfg.pairing_queue)
    sent: deque = deque(maxlen=cfg.pairing_queue)
    mean_hist: deque = deque(maxlen=cfg.smoothing_window)
    max_hist: deque = deque(maxlen=cfg.smoothing_window)
    records: List[dict] = []
    if save_dir:
        os.makedirs(save_dir, exist_ok=True)
    try:
        with grpc.insecure_channel(cfg.server_address) as channel:
            stub = pb.VisionAnalysisServiceStub(channel)
            for resp in stub.AnalyzeActuatorPerformance(generate_requests(cam, frame_queue, max_frames, None, sent)):
                t_now = time.perf_counter()
                if not frame_queue:
                    continue
                color = frame_queue.popleft()
                rtt = (t_now - sent.popleft()) * 1e3 if sent else float("nan")
                mean_hist.append(resp.mean_curvature)
                max_hist.append(resp.max_curvature)
                rec = dict(mean_curvature=resp.mean_curvature, max_curvature=resp.max_curvature, status=resp.status,
                           mask_coverage=resp.mask_coverage, proc_time_ms=resp.proc_time_ms, rtt_ms=rtt,
                           smoothed_mean=float(np.mean(mean_hist)), smoothed_max=float(np.mean(max_hist)),
                           n_spline=len(resp.spline_points))
                records.append(rec)
                if render or save_dir:
                    img = render_overlay(color, resp, K, dist)
                    if save_dir:
                        imwrite(os.path.join(save_dir, f"frame_{len(records):05d}.png"), img)
    except grpc.RpcError as e:
        log.error("could not reach server: %s", e.details() if hasattr(e, "details") else e)
    finally:
        if own_cam:
            cam.stop()
    return records

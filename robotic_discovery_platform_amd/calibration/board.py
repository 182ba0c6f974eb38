"""Checkerboard geometry and a synthetic renderer (pinhole + Brown distortion, supersampled).

``object_points`` follows the reference's grid construction (``scripts/01_calibrate_camera.py:43-45``:
``objp[:, :2] = mgrid[0:9, 0:7].T.reshape(-1, 2) * square``): row-major with the first pattern
dimension varying fastest, z = 0.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from .zhang import project_points, rodrigues


def object_points(pattern: Tuple[int, int] = (9, 7), square: float = 0.027) -> np.ndarray:
    nx, ny = pattern
    objp = np.zeros((nx * ny, 3), np.float32)
    objp[:, :2] = np.mgrid[0:nx, 0:ny].T.reshape(-1, 2) * square
    return objp


def _undistort_normalized(xd: np.ndarray, yd: np.ndarray, d: np.ndarray, iters: int = 12):
    k1, k2, p1, p2, k3 = d
    x, y = xd.copy(), yd.copy()
    for _ in range(iters):
        r2 = x * x + y * y
        radial = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 ** 3
        dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
        dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
        x = (xd - dx) / radial
        y = (yd - dy) / radial
    return x, y


def render_board_view(K: np.ndarray, dist: Optional[np.ndarray], rvec, tvec, pattern=(9, 7), square=0.027,
                      size=(640, 480), ss: int = 3, noise: float = 2.0, seed: int = 0) -> np.ndarray:
    """Grayscale uint8 image of the board (pattern+1 squares per side, one white square margin)."""
    W, H = size
    nx, ny = pattern
    d = np.zeros(5) if dist is None else np.pad(np.asarray(dist, np.float64).ravel(), (0, 5))[:5]
    R = rodrigues(np.asarray(rvec, np.float64).reshape(3))
    t = np.asarray(tvec, np.float64).reshape(3)
    Hinv = np.linalg.inv(np.stack([R[:, 0], R[:, 1], t], 1))
    o = (np.arange(ss) + 0.5) / ss - 0.5
    u = (np.arange(W)[None, :, None, None] + o[None, None, None, :])
    v = (np.arange(H)[:, None, None, None] + o[None, None, :, None])
    u, v = np.broadcast_arrays(u, v)
    xd = (u - K[0, 2]) / K[0, 0]
    yd = (v - K[1, 2]) / K[1, 1]
    x, y = _undistort_normalized(xd, yd, d)
    q = np.stack([x, y, np.ones_like(x)], -1) @ Hinv.T
    X, Y = q[..., 0] / q[..., 2], q[..., 1] / q[..., 2]
    front = q[..., 2] > 0
    ix = np.floor(X / square).astype(np.int64)
    iy = np.floor(Y / square).astype(np.int64)
    on_sq = (ix >= -1) & (ix <= nx - 1) & (iy >= -1) & (iy <= ny - 1)
    on_margin = (X >= -2 * square) & (X <= (nx + 1) * square) & (Y >= -2 * square) & (Y <= (ny + 1) * square)
    black = ((ix + iy) % 2 == 0) & on_sq
    img = np.full(X.shape, 95.0)
    img = np.where(front & on_margin, 235.0, img)
    img = np.where(front & black, 25.0, img)
    img = img.mean(axis=(2, 3))
    rng = np.random.default_rng(seed)
    img = img + rng.normal(0, noise, img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def random_board_pose(rng: np.random.Generator, K: np.ndarray, pattern=(9, 7), square=0.027, size=(640, 480),
                      dist=None, margin: float = 40.0, max_tilt_deg: float = 35.0):
    """A pose (rvec, tvec) with the whole board (incl. margin squares) inside the image."""
    W, H = size
    nx, ny = pattern
    corners = np.array([[-2, -2, 0], [nx + 1, -2, 0], [nx + 1, ny + 1, 0], [-2, ny + 1, 0]], np.float64) * square
    for _ in range(1000):
        ang = np.deg2rad(rng.uniform(-max_tilt_deg, max_tilt_deg, 2))
        rz = np.deg2rad(rng.uniform(-20, 20))
        R = rodrigues(np.array([ang[0], 0, 0])) @ rodrigues(np.array([0, ang[1], 0])) @ rodrigues(np.array([0, 0, rz]))
        z = rng.uniform(0.35, 0.6)
        c = np.array([(nx - 1) / 2 * square, (ny - 1) / 2 * square, 0])
        off = np.array([rng.uniform(-0.06, 0.06), rng.uniform(-0.04, 0.04), z])
        t = off - R @ c
        rvec = rodrigues(R)
        p = project_points(corners, rvec, t, K, dist)
        if (p[:, 0].min() > margin and p[:, 0].max() < W - margin and p[:, 1].min() > margin
                and p[:, 1].max() < H - margin):
            return rvec, t
    raise RuntimeError("no valid board pose found")

"""Synthetic RGB-D soft-actuator scenes (there is no camera, dataset or network in this environment).

A scene is what the reference's RealSense pipeline delivers (``/root/reference/pkg/camera.py:35,62-63``):
a 640x480 uint8 BGR colour frame, a 640x480 uint16 z16 depth frame aligned to colour (units of
``depth_scale`` metres), plus the ground-truth segmentation mask and the analytic bend curvature
of the actuator, so the geometry pipeline has a known answer.

The actuator is a circular-arc band of radius R (curvature 1/R) lying on a tilted plane; its
lower edge (largest image y) is the edge the reference curvature path tracks
(``pkg/geometry_utils.py:119-142``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

DEFAULT_K = np.array([[615.0, 0.0, 320.0], [0.0, 615.0, 240.0], [0.0, 0.0, 1.0]])


@dataclass
class Scene:
    color: np.ndarray  # HxWx3 uint8 BGR
    depth: np.ndarray  # HxW uint16 (depth_scale units)
    mask: np.ndarray  # HxW uint8 {0, 255}
    curvature: float  # analytic curvature of the actuator centre line (1/m)
    radius_m: float


def make_scene(seed: int = 0, width: int = 640, height: int = 480, K: np.ndarray = DEFAULT_K,
               depth_scale: float = 0.001, radius_m: Optional[float] = None, thickness_m: float = 0.012,
               arc_deg: Optional[float] = None, z0: Optional[float] = None, noise: float = 4.0) -> Scene:
    rng = np.random.default_rng(seed)
    R = radius_m if radius_m is not None else float(rng.uniform(0.06, 0.15))
    arc = np.deg2rad(arc_deg if arc_deg is not None else float(rng.uniform(50, 100)))
    z0 = z0 if z0 is not None else float(rng.uniform(0.45, 0.65))
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    # arc in the camera's x-y plane at depth ~z0, opening downwards (bending actuator)
    cx_w = float(rng.uniform(-0.02, 0.02))
    cy_w = float(rng.uniform(-0.02, 0.03)) - R  # lowest point of the arc near the image centre
    vv, uu = np.mgrid[0:height, 0:width]
    # back-project every pixel onto the plane z = z0 + tilt*y
    tilt = float(rng.uniform(-0.15, 0.15))
    # ray: X = (u-cx)/fx * Z, Y = (v-cy)/fy * Z, plane Z = z0 + tilt*Y  => Z = z0 / (1 - tilt*(v-cy)/fy)
    Z = z0 / (1.0 - tilt * (vv - cy) / fy)
    X = (uu - cx) / fx * Z
    Y = (vv - cy) / fy * Z
    dx, dy = X - cx_w, Y - cy_w
    r = np.hypot(dx, dy)
    ang = np.arctan2(dy, dx)
    # angular window centred on pi/2 (pointing +y, i.e. down in the image) of width `arc`
    d_ang = np.angle(np.exp(1j * (ang - np.pi / 2)))
    band = (np.abs(r - R) < thickness_m / 2) & (np.abs(d_ang) < arc / 2)
    mask = band.astype(np.uint8) * 255
    # depth: background plane slightly behind, actuator raised towards the camera
    depth_m = Z + 0.05
    depth_m = np.where(band, Z - 0.01 * np.cos(np.clip((r - R) / thickness_m * np.pi, -np.pi / 2, np.pi / 2)),
                       depth_m)
    depth_m = depth_m + rng.normal(0, 0.0005, depth_m.shape)
    # a few invalid (zero) depth pixels like a real z16 stream
    holes = rng.random(depth_m.shape) < 0.002
    depth = np.where(holes, 0, np.round(depth_m / depth_scale)).astype(np.uint16)
    # colour: textured grey background, reddish actuator with shading
    base = 110 + 25 * np.sin(uu / 37.0) * np.cos(vv / 53.0)
    color = np.stack([base, base + 5, base - 5], -1)
    shade = 0.75 + 0.25 * np.cos(d_ang * 2)
    act = np.stack([40 * shade, 60 * shade, 200 * shade], -1)  # BGR: red actuator
    color = np.where(band[..., None], act, color)
    color = color + rng.normal(0, noise, color.shape)
    color = np.clip(np.rint(color), 0, 255).astype(np.uint8)
    return Scene(color=color, depth=depth, mask=mask, curvature=1.0 / R, radius_m=R)


def make_batch(n: int, size: Tuple[int, int] = (256, 256), seed: int = 0):
    """(images float [n,3,H,W] in [0,1] RGB, masks float [n,1,H,W]) resized like the trainer does."""
    from .image_io import bgr2rgb, resize_area, resize_nearest
    imgs, masks = [], []
    for i in range(n):
        s = make_scene(seed + i)
        imgs.append(resize_area(bgr2rgb(s.color), size).astype(np.float32) / 255.0)
        masks.append(resize_nearest(s.mask, size).astype(np.float32) / 255.0)
    x = np.stack(imgs).transpose(0, 3, 1, 2)
    y = np.stack(masks)[:, None]
    return x, y


def write_dataset(root: str, n: int, seed: int = 0, fmt: str = "png") -> int:
    """Materialise ``n`` scenes as ml/datasets/processed/{images,masks}/<name> (paired by filename)."""
    import os
    from .image_io import imwrite
    img_dir, mask_dir = os.path.join(root, "images"), os.path.join(root, "masks")
    os.makedirs(img_dir, exist_ok=True)
    os.makedirs(mask_dir, exist_ok=True)
    for i in range(n):
        s = make_scene(seed + i)
        name = f"scene_{seed + i:05d}.{fmt}"
        imwrite(os.path.join(img_dir, name), s.color)
        imwrite(os.path.join(mask_dir, name), s.mask)
    return n


def auto_label(depth: np.ndarray, depth_scale: float = 0.001, margin_m: float = 0.02,
               min_valid_frac: float = 0.5) -> np.ndarray:
    """Depth-threshold auto-labeller for collected raw frames (the reference README promises
    "collect and auto-label" but ships no labeller): pixels noticeably closer than the
    per-row background depth (median) are foreground. Returns a {0,255} uint8 mask."""
    d = depth.astype(np.float64) * depth_scale
    valid = d > 0
    bg = np.where(valid, d, np.nan)
    row_med = np.nanmedian(bg, axis=1, keepdims=True)
    fg = valid & (d < row_med - margin_m)
    return (fg.astype(np.uint8) * 255)

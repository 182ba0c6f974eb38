"""NumPy/SciPy oracle of the reference curvature pipeline (tests only; never the serving path).

Semantics of ``/root/reference/pkg/geometry_utils.py:42-162``:
  1. point cloud: pixels with mask > 0 in row-major order, z = depth*scale, keep z > 0,
     x = (u-cx) z / fx, y = (v-cy) z / fy (float64)                                    (:101-117)
  2. < 100 points -> empty result                                                      (:64-65)
  3. edge: < num_bins points -> none; bin by x into 50 bins of width (max-min)/50 (none if
     width <= 0), idx = clip(floor((x-min)/w), 0, 49); per non-empty bin keep the top
     k = max(1, int(n*0.05)) points by largest y                                        (:119-142)
  4. < 20 edge points -> empty                                                          (:69-70)
  5. sort by x, ``splprep([x,y,z], s=0.1, k=3)``, curvature |r'xr''|/|r'|^3 over 100 samples
     where |r'| > 1e-6 (mean, max), 100 spline points at u = linspace(0,1,100)           (:74-97,144-162)
  6. TypeError / ValueError from the fit -> empty result                                 (:95-97)
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

import numpy as np


@dataclass
class Point:
    x: float = 0.0
    y: float = 0.0
    z: float = 0.0


@dataclass
class CurvatureResult:
    mean_curvature: float = 0.0
    max_curvature: float = 0.0
    spline_points: List[Point] = field(default_factory=list)
    status: str = "ok"


def point_cloud(mask, depth, K, scale):
    v, u = np.nonzero(mask > 0)
    z = depth[v, u].astype(np.float64) * scale
    keep = z > 0
    v, u, z = v[keep], u[keep], z[keep]
    x = (u - K[0, 2]) * z / K[0, 0]
    y = (v - K[1, 2]) * z / K[1, 1]
    return np.stack([x, y, z], 1)


def edge_points(pcd, num_bins=50, top=0.05):
    if pcd.shape[0] < num_bins:
        return np.zeros((0, 3))
    lo, hi = pcd[:, 0].min(), pcd[:, 0].max()
    width = (hi - lo) / num_bins
    if width <= 0:
        return np.zeros((0, 3))
    idx = np.clip(np.floor((pcd[:, 0] - lo) / width).astype(int), 0, num_bins - 1)
    out = []
    for b in range(num_bins):
        sel = pcd[idx == b]
        if len(sel):
            k = max(1, int(len(sel) * top))
            out.append(sel[np.argsort(-sel[:, 1], kind="stable")[:k]])
    return np.concatenate(out) if out else np.zeros((0, 3))


def spline_curvature(tck, n=100, eps=1e-6):
    from scipy.interpolate import splev
    u = np.linspace(0, 1, n)
    d1 = np.array(splev(u, tck, der=1)).T
    d2 = np.array(splev(u, tck, der=2)).T
    num = np.linalg.norm(np.cross(d1, d2), axis=1)
    den = np.linalg.norm(d1, axis=1)
    ok = den > eps
    if not ok.any():
        return 0.0, 0.0
    kap = num[ok] / den[ok] ** 3
    return float(kap.mean()), float(kap.max())


def compute_curvature_profile(mask, depth, K, scale, s=0.1, k=3, min_points=100, min_edge=20):
    from scipy.interpolate import splev, splprep
    pcd = point_cloud(mask, depth, K, scale)
    if pcd.shape[0] < min_points:
        return CurvatureResult(status="too_few_points")
    e = edge_points(pcd)
    if e.shape[0] < min_edge:
        return CurvatureResult(status="too_few_edge_points")
    e = e[np.argsort(e[:, 0], kind="stable")]
    try:
        tck, _ = splprep([e[:, 0], e[:, 1], e[:, 2]], s=s, k=k)
    except (TypeError, ValueError):
        return CurvatureResult(status="fit_failed")
    mk, xk = spline_curvature(tck)
    pts = np.array(splev(np.linspace(0, 1, 100), tck)).T
    return CurvatureResult(mk, xk, [Point(*map(float, p)) for p in pts])

"""Checkerboard inner-corner detection and sub-pixel refinement.

``find_chessboard_corners(gray, pattern)`` -> ``(found, corners[N,1,2] float32)`` and
``corner_subpix(gray, corners, win, max_iter, eps)`` mirror the two OpenCV calls of
``/root/reference/scripts/01_calibrate_camera.py:78-90``.

Detector: X-corners are saddle points of the smoothed intensity, where the Hessian determinant is
strongly negative; candidates are local maxima of ``-det(H)``. The grid is recovered by fitting a
homography from the ideal (nx, ny) lattice to the candidates: the lattice's four outer corners
are tried against every 4-vertex subset of the candidates' convex hull, the projected lattice is
matched to the nearest candidates, and the homography is re-fitted on the matches (absorbing
moderate lens distortion). The order is row-major with ``pattern[0]`` points per row; of the two
orientations a symmetric pattern admits, the one whose first corner is nearest the image origin
is returned (non-mirrored only).

Sub-pixel refinement solves the classic orthogonality condition: for pixels p in the window
around q, the image gradient g(p) is orthogonal to (p - q) at a true corner, so
q = (sum w g g^T)^-1 sum w g g^T p, iterated until the update is below ``eps``.
"""
from __future__ import annotations

from itertools import combinations
from typing import Optional, Tuple

import numpy as np


def _saddle_candidates(gray: np.ndarray, sigma: float, max_cand: int):
    from scipy import ndimage as ndi
    g = gray.astype(np.float64)
    Ixx = ndi.gaussian_filter(g, sigma, order=(0, 2))
    Iyy = ndi.gaussian_filter(g, sigma, order=(2, 0))
    Ixy = ndi.gaussian_filter(g, sigma, order=(1, 1))
    R = -(Ixx * Iyy - Ixy * Ixy)
    R[R < 0] = 0
    r = max(3, int(round(2 * sigma)))
    mx = ndi.maximum_filter(R, size=2 * r + 1)
    b = int(np.ceil(3 * sigma))
    peak = (R == mx) & (R > 0.08 * R.max())
    peak[:b], peak[-b:], peak[:, :b], peak[:, -b:] = False, False, False, False
    ys, xs = np.nonzero(peak)
    vals = R[ys, xs]
    o = np.argsort(-vals)[:max_cand]
    pts = np.stack([xs[o], ys[o]], 1).astype(np.float64)
    # sub-pixel peak (quadratic fit of the response)
    for k, (x, y) in enumerate(pts.astype(int)):
        if 0 < x < R.shape[1] - 1 and 0 < y < R.shape[0] - 1:
            dx = (R[y, x + 1] - R[y, x - 1]) / 2
            dy = (R[y + 1, x] - R[y - 1, x]) / 2
            dxx = R[y, x + 1] - 2 * R[y, x] + R[y, x - 1]
            dyy = R[y + 1, x] - 2 * R[y, x] + R[y - 1, x]
            if dxx < 0 and dyy < 0:
                pts[k] += [np.clip(-dx / dxx, -0.5, 0.5), np.clip(-dy / dyy, -0.5, 0.5)]
    return pts, vals[o]


def _homog(src, dst):
    from .zhang import _homography
    return _homography(src, dst)


def _apply(H, p):
    q = np.c_[p, np.ones(len(p))] @ H.T
    return q[:, :2] / q[:, 2:3]


def _match(grid_px, tree, ncand, tol):
    d, i = tree.query(grid_px)
    ok = d < tol
    if len(np.unique(i[ok])) != ok.sum():  # two lattice points on one candidate: reject duplicates
        ok &= np.bincount(i, minlength=ncand)[i] == 1
    return ok, i


def find_chessboard_corners(gray: np.ndarray, pattern: Tuple[int, int] = (9, 7), sigma: Optional[float] = None):
    from scipy.spatial import ConvexHull, cKDTree
    nx, ny = pattern
    N = nx * ny
    if gray.ndim == 3:
        gray = gray[..., :3].mean(-1)
    sigma = sigma or max(1.5, min(gray.shape) / 320.0)
    cand, vals = _saddle_candidates(gray, sigma, 4 * N)
    if len(cand) < N:
        return False, None
    # X-junctions respond far more strongly than T/L junctions at the board border: keep the
    # candidates within a fraction of the typical response of the N strongest
    cand = cand[vals > 0.3 * np.median(vals[:N])]
    if len(cand) < N:
        return False, None
    lattice = np.mgrid[0:nx, 0:ny].T.reshape(-1, 2).astype(np.float64)  # row-major, x fastest
    outer = np.array([[0, 0], [nx - 1, 0], [nx - 1, ny - 1], [0, ny - 1]], np.float64)
    try:
        hull = cand[ConvexHull(cand).vertices]
    except Exception:
        return False, None
    tree = cKDTree(cand)
    if len(hull) > 10:  # keep the most "cornery" hull vertices (sharpest turns)
        prv, nxt = np.roll(hull, 1, 0), np.roll(hull, -1, 0)
        a, b = prv - hull, nxt - hull
        cosang = (a * b).sum(1) / (np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1) + 1e-12)
        hull = hull[np.sort(np.argsort(cosang)[-10:])]
    best = None
    for quad_idx in combinations(range(len(hull)), 4):
        quad = hull[list(quad_idx)]
        for rot in range(4):
            q = np.roll(quad, rot, 0)
            for flip in (False, True):
                qq = q[::-1] if flip else q
                try:
                    H = _homog(outer, qq)
                except np.linalg.LinAlgError:
                    continue
                px = _apply(H, lattice)
                spacing = np.median(np.linalg.norm(px[1:nx] - px[:nx - 1], axis=1))
                if not np.isfinite(spacing) or spacing < 3:
                    continue
                ok, idx = _match(px, tree, len(cand), 0.3 * spacing)
                if ok.sum() < N // 2:
                    continue
                for _ in range(3):  # re-fit on matches to absorb distortion
                    H = _homog(lattice[ok], cand[idx[ok]])
                    px = _apply(H, lattice)
                    ok, idx = _match(px, tree, len(cand), 0.3 * spacing)
                    if ok.sum() == N or ok.sum() < 8:
                        break
                score = ok.sum()
                if score == N:
                    pts = cand[idx]
                    e1, e2 = pts[1] - pts[0], pts[nx] - pts[0]
                    if e1[0] * e2[1] - e1[1] * e2[0] <= 0:  # mirrored lattice
                        continue
                    key = pts[0].sum()
                    if best is None or key < best[0] - 1e-6:
                        best = (key, pts.copy())
    if best is None:
        return False, None
    return True, best[1].reshape(-1, 1, 2).astype(np.float32)


def _bilinear(img: np.ndarray, x: np.ndarray, y: np.ndarray) -> np.ndarray:
    H, W = img.shape
    x = np.clip(x, 0, W - 1.001)
    y = np.clip(y, 0, H - 1.001)
    x0, y0 = np.floor(x).astype(int), np.floor(y).astype(int)
    fx, fy = x - x0, y - y0
    return (img[y0, x0] * (1 - fx) * (1 - fy) + img[y0, x0 + 1] * fx * (1 - fy) + img[y0 + 1, x0] * (1 - fx) * fy
            + img[y0 + 1, x0 + 1] * fx * fy)


def corner_subpix(gray: np.ndarray, corners: np.ndarray, win: Tuple[int, int] = (11, 11), max_iter: int = 30,
                  eps: float = 0.001) -> np.ndarray:
    """Refine corners in place-like fashion; ``win`` is the half window (OpenCV convention)."""
    g = gray.astype(np.float64)
    if g.ndim == 3:
        g = g[..., :3].mean(-1)
    gy, gx = np.gradient(g)
    wx, wy = win
    ox, oy = np.meshgrid(np.arange(-wx, wx + 1, dtype=np.float64), np.arange(-wy, wy + 1, dtype=np.float64))
    ox, oy = ox.ravel(), oy.ravel()
    wgt = np.exp(-(ox ** 2 / (wx * wx) + oy ** 2 / (wy * wy)))  # OpenCV-like Gaussian window weights
    out = np.asarray(corners, np.float64).reshape(-1, 2).copy()
    for k in range(len(out)):
        q = out[k].copy()
        for _ in range(max_iter):
            px, py = q[0] + ox, q[1] + oy
            ax, ay = _bilinear(gx, px, py), _bilinear(gy, px, py)
            a11, a12, a22 = (wgt * ax * ax).sum(), (wgt * ax * ay).sum(), (wgt * ay * ay).sum()
            b1 = (wgt * (ax * ax * px + ax * ay * py)).sum()
            b2 = (wgt * (ax * ay * px + ay * ay * py)).sum()
            det = a11 * a22 - a12 * a12
            if abs(det) < 1e-12:
                break
            qn = np.array([(a22 * b1 - a12 * b2) / det, (a11 * b2 - a12 * b1) / det])
            moved = np.linalg.norm(qn - q)
            if np.linalg.norm(qn - out[k]) > max(wx, wy):  # diverged out of the window
                break
            q = qn
            if moved < eps:
                break
        out[k] = q
    return out.reshape(-1, 1, 2).astype(np.float32)

"""Zhang's planar calibration with Brown-Conrady distortion (k1, k2, p1, p2, k3).

``calibrate_camera(object_points, image_points, image_size)`` returns ``(rms, mtx, dist, rvecs,
tvecs)`` with the shapes of ``cv2.calibrateCamera`` (the reference call at
``/root/reference/scripts/01_calibrate_camera.py:100``): initial K from the homography constraints
(closed form), per-view extrinsics from K^-1 H, then joint Levenberg-Marquardt refinement of all
intrinsics, distortion and poses over the reprojection residuals (scipy ``least_squares``).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def rodrigues(v: np.ndarray) -> np.ndarray:
    """Rotation vector <-> matrix (like cv2.Rodrigues): (3,) -> (3,3) or (3,3) -> (3,)."""
    v = np.asarray(v, np.float64)
    if v.shape == (3, 3):
        R = v
        c = np.clip((np.trace(R) - 1) / 2, -1.0, 1.0)
        th = np.arccos(c)
        if th < 1e-12:
            return np.zeros(3)
        if np.pi - th < 1e-6:  # ~180 deg: axis from the symmetric part
            w, V = np.linalg.eigh((R + np.eye(3)) / 2)
            ax = V[:, np.argmax(w)]
            return ax * th
        ax = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]]) / (2 * np.sin(th))
        return ax * th
    v = v.reshape(3)
    th = np.linalg.norm(v)
    if th < 1e-12:
        return np.eye(3)
    k = v / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def _distort(x: np.ndarray, y: np.ndarray, d: np.ndarray):
    k1, k2, p1, p2, k3 = d
    r2 = x * x + y * y
    radial = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 ** 3
    xd = x * radial + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * radial + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return xd, yd


def project_points(obj: np.ndarray, rvec, tvec, K: np.ndarray, dist=None) -> np.ndarray:
    """cv2.projectPoints equivalent: (N,3) world points -> (N,2) pixels."""
    obj = np.asarray(obj, np.float64).reshape(-1, 3)
    R = rodrigues(np.asarray(rvec, np.float64).reshape(3))
    P = obj @ R.T + np.asarray(tvec, np.float64).reshape(1, 3)
    z = np.where(np.abs(P[:, 2]) > 1e-12, P[:, 2], 1e-12)
    x, y = P[:, 0] / z, P[:, 1] / z
    d = np.zeros(5) if dist is None else np.pad(np.asarray(dist, np.float64).ravel(), (0, 5))[:5]
    xd, yd = _distort(x, y, d)
    return np.stack([K[0, 0] * xd + K[0, 1] * yd + K[0, 2], K[1, 1] * yd + K[1, 2]], 1)


def _homography(src: np.ndarray, dst: np.ndarray) -> np.ndarray:
    """Normalised DLT: src (N,2) plane coords -> dst (N,2) pixels."""
    def norm(p):
        c = p.mean(0)
        s = np.sqrt(2) / np.mean(np.linalg.norm(p - c, axis=1))
        T = np.array([[s, 0, -s * c[0]], [0, s, -s * c[1]], [0, 0, 1]])
        return T, (p - c) * s

    Ts, s = norm(src)
    Td, d = norm(dst)
    A = []
    for (x, y), (u, v) in zip(s, d):
        A.append([-x, -y, -1, 0, 0, 0, u * x, u * y, u])
        A.append([0, 0, 0, -x, -y, -1, v * x, v * y, v])
    _, _, Vt = np.linalg.svd(np.asarray(A))
    Hn = Vt[-1].reshape(3, 3)
    H = np.linalg.inv(Td) @ Hn @ Ts
    return H / H[2, 2]


def _v(H, i, j):
    h = H.T
    return np.array([h[i, 0] * h[j, 0], h[i, 0] * h[j, 1] + h[i, 1] * h[j, 0], h[i, 1] * h[j, 1],
                     h[i, 2] * h[j, 0] + h[i, 0] * h[j, 2], h[i, 2] * h[j, 1] + h[i, 1] * h[j, 2], h[i, 2] * h[j, 2]])


def _init_intrinsics(Hs: Sequence[np.ndarray], image_size: Tuple[int, int]) -> np.ndarray:
    W, H = image_size
    if len(Hs) >= 3:
        V = np.concatenate([[_v(Hk, 0, 1), _v(Hk, 0, 0) - _v(Hk, 1, 1)] for Hk in Hs])
        _, _, Vt = np.linalg.svd(V)
        B11, B12, B22, B13, B23, B33 = Vt[-1]
        v0 = (B12 * B13 - B11 * B23) / (B11 * B22 - B12 * B12)
        lam = B33 - (B13 * B13 + v0 * (B12 * B13 - B11 * B23)) / B11
        with np.errstate(invalid="ignore"):
            fx = np.sqrt(lam / B11)
            fy = np.sqrt(lam * B11 / (B11 * B22 - B12 * B12))
        u0 = -B13 * fx * fx / lam
        if np.all(np.isfinite([fx, fy, u0, v0])) and fx > 0 and fy > 0 and 0 < u0 < W and 0 < v0 < H:
            return np.array([[fx, 0, u0], [0, fy, v0], [0, 0, 1.0]])
    # fall back: principal point at the centre, focal from the vanishing-point constraint
    cx, cy = (W - 1) / 2, (H - 1) / 2
    T = np.array([[1, 0, -cx], [0, 1, -cy], [0, 0, 1.0]])
    f2 = []
    for Hk in Hs:
        h = T @ Hk
        a = -(h[0, 0] * h[0, 1] + h[1, 0] * h[1, 1]) / max(h[2, 0] * h[2, 1], 1e-12) if abs(h[2, 0] * h[2, 1]) > 1e-12 else None
        if a is not None and a > 0:
            f2.append(a)
    f = np.sqrt(np.median(f2)) if f2 else max(W, H)
    return np.array([[f, 0, cx], [0, f, cy], [0, 0, 1.0]])


def _extrinsics(Hk: np.ndarray, K: np.ndarray):
    Ki = np.linalg.inv(K)
    h1, h2, h3 = Hk[:, 0], Hk[:, 1], Hk[:, 2]
    lam = 1.0 / np.linalg.norm(Ki @ h1)
    r1, r2 = lam * Ki @ h1, lam * Ki @ h2
    t = lam * Ki @ h3
    if t[2] < 0:  # board in front of the camera
        r1, r2, t = -r1, -r2, -t
    R = np.stack([r1, r2, np.cross(r1, r2)], 1)
    U, _, Vt = np.linalg.svd(R)
    R = U @ Vt
    if np.linalg.det(R) < 0:
        R = U @ np.diag([1, 1, -1]) @ Vt
    return rodrigues(R), t


def reprojection_errors(obj_pts, img_pts, K, dist, rvecs, tvecs) -> List[float]:
    """Per-view mean L2 reprojection error (the reference's report, 01_calibrate_camera.py:107-112)."""
    out = []
    for o, i, r, t in zip(obj_pts, img_pts, rvecs, tvecs):
        p = project_points(o, r, t, K, dist)
        out.append(float(np.linalg.norm(p - np.asarray(i).reshape(-1, 2), axis=1).mean()))
    return out


def calibrate_camera(object_points: Sequence[np.ndarray], image_points: Sequence[np.ndarray],
                     image_size: Tuple[int, int], fix_k3: bool = False, max_nfev: int = 200):
    """(rms, mtx[3,3], dist[1,5], rvecs list of (3,1), tvecs list of (3,1)); image_size = (W, H)."""
    from scipy.optimize import least_squares
    objs = [np.asarray(o, np.float64).reshape(-1, 3) for o in object_points]
    imgs = [np.asarray(i, np.float64).reshape(-1, 2) for i in image_points]
    if len(objs) < 1 or any(o.shape[0] < 4 for o in objs):
        raise ValueError("need at least one view with >= 4 points")
    if any(np.abs(o[:, 2]).max() > 1e-9 for o in objs):
        raise ValueError("planar calibration: object points must have z == 0")
    Hs = [_homography(o[:, :2], i) for o, i in zip(objs, imgs)]
    K0 = _init_intrinsics(Hs, image_size)
    poses = [_extrinsics(Hk, K0) for Hk in Hs]
    nv = len(objs)

    def unpack(x):
        K = np.array([[x[0], 0, x[2]], [0, x[1], x[3]], [0, 0, 1.0]])
        d = x[4:9].copy()
        if fix_k3:
            d[4] = 0
        return K, d, x[9:].reshape(nv, 6)

    def resid(x):
        K, d, P = unpack(x)
        r = [project_points(o, P[k, :3], P[k, 3:], K, d) - i for k, (o, i) in enumerate(zip(objs, imgs))]
        return np.concatenate(r).ravel()

    x0 = np.concatenate([[K0[0, 0], K0[1, 1], K0[0, 2], K0[1, 2]], np.zeros(5),
                         np.concatenate([np.r_[r, t] for r, t in poses])])
    # stage 1: pinhole only (distortion frozen at 0) for a stable basin, stage 2: everything
    free = np.ones_like(x0, bool)
    free[4:9] = False

    def resid_sub(xs, mask, base):
        x = base.copy()
        x[mask] = xs
        return resid(x)

    s1 = least_squares(resid_sub, x0[free], args=(free, x0), method="lm", max_nfev=max_nfev * len(x0))
    x1 = x0.copy()
    x1[free] = s1.x
    free2 = np.ones_like(x0, bool)
    if fix_k3:
        free2[8] = False
    s2 = least_squares(resid_sub, x1[free2], args=(free2, x1), method="lm", max_nfev=max_nfev * len(x0))
    x2 = x1.copy()
    x2[free2] = s2.x
    K, d, P = unpack(x2)
    r = resid(x2).reshape(-1, 2)
    rms = float(np.sqrt((r ** 2).sum(1).mean()))
    rvecs = [P[k, :3].reshape(3, 1) for k in range(nv)]
    tvecs = [P[k, 3:].reshape(3, 1) for k in range(nv)]
    return rms, K, d.reshape(1, 5), rvecs, tvecs

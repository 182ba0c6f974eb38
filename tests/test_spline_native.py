"""Native FITPACK-equivalent parametric smoothing spline vs scipy.interpolate.splprep/splev (CPU)."""
import numpy as np
import pytest
import torch
from scipy.interpolate import splev, splprep

from robotic_discovery_platform_amd.ops import native


def _chord(p):
    d = np.r_[0, np.cumsum(np.linalg.norm(np.diff(p, axis=0), axis=1))]
    return d / d[-1]


def _case(kind, seed):
    rng = np.random.default_rng(seed)
    m = int(rng.integers(25, 400))
    th = np.sort(rng.uniform(0, 1.6, m))
    R = rng.uniform(0.05, 0.3)
    x = R * np.sin(th)
    y = R * (1 - np.cos(th))
    z = 0.5 + 0.02 * th
    noise = {"smooth": 0.0005, "noisy": 0.02, "wild": 0.08}[kind]
    p = np.stack([x, y, z], 1) + rng.normal(0, noise, (m, 3))
    p = p[np.argsort(p[:, 0], kind="stable")]
    return p


@pytest.mark.parametrize("kind", ["smooth", "noisy", "wild"])
@pytest.mark.parametrize("s", [0.1, 0.01, 0.001])
@pytest.mark.parametrize("seed", range(4))
def test_parcur_matches_scipy(kind, s, seed):
    C = native()
    p = _case(kind, seed)
    u = _chord(p)
    ier, t, c, fp = C.parcur(torch.from_numpy(u), torch.from_numpy(np.ascontiguousarray(p)), s, 3)
    ((tr, cr, kr), ur), fpr, ierr, _ = splprep([p[:, 0], p[:, 1], p[:, 2]], u=u, s=s, k=3, full_output=True, quiet=1)
    assert np.allclose(ur, u)
    assert ier == ierr
    assert t.numel() == len(tr) and np.allclose(t.numpy(), tr, atol=1e-12)
    uu = np.linspace(0, 1, 57)
    for j in range(3):
        for der in (0, 1, 2):
            ref = splev(uu, (tr, cr[j], 3), der=der)
            got = C.splev(t, c[j].contiguous(), 3, torch.from_numpy(uu), der).numpy()
            scale = np.abs(ref).max() + 1e-9
            assert np.abs(got - ref).max() / scale < 1e-6, (j, der)
    assert fp == pytest.approx(fpr, rel=1e-6, abs=1e-12)


def test_fit_curvature_matches_reference_math():
    C = native()
    p = _case("smooth", 7)
    ier, mk, xk, pts, fp, n = C.fit_curvature(torch.from_numpy(np.ascontiguousarray(p)), 0.1, 3, 100, 1e-6)
    tck, _ = splprep([p[:, 0], p[:, 1], p[:, 2]], s=0.1, k=3)
    from robotic_discovery_platform_amd.geometry.reference import spline_curvature
    rm, rx = spline_curvature(tck)
    assert mk == pytest.approx(rm, rel=1e-7) and xk == pytest.approx(rx, rel=1e-7)
    ref_pts = np.array(splev(np.linspace(0, 1, 100), tck)).T
    assert np.abs(pts.numpy() - ref_pts).max() < 1e-9


def test_fit_invalid_input():
    C = native()
    ier = C.fit_curvature(torch.zeros(3, 3, dtype=torch.float64), 0.1, 3, 100, 1e-6)[0]
    assert ier == 10

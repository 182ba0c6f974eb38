"""Curvature pipeline (CPU path: numpy edge extraction + native C++ spline) vs the scipy oracle.

Oracle = geometry/reference.py, which restates /root/reference/pkg/geometry_utils.py:42-162.
"""
import numpy as np
import pytest

from robotic_discovery_platform_amd.config import GeometryConfig
from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K, make_scene
from robotic_discovery_platform_amd.geometry import reference as ref
from robotic_discovery_platform_amd.geometry.curvature import compute_curvature_profile, edges_numpy, sort_edges


@pytest.mark.parametrize("seed", range(6))
def test_edges_match_oracle(seed):
    sc = make_scene(seed)
    e, n = edges_numpy(sc.mask, sc.depth, DEFAULT_K, 0.001, GeometryConfig())
    pcd = ref.point_cloud(sc.mask, sc.depth, DEFAULT_K, 0.001)
    assert n == pcd.shape[0]
    eo = ref.edge_points(pcd)
    eo = eo[np.argsort(eo[:, 0], kind="stable")]
    assert np.array_equal(sort_edges(e), eo)


@pytest.mark.parametrize("seed", range(6))
def test_curvature_matches_oracle(seed):
    sc = make_scene(seed)
    got = compute_curvature_profile(sc.mask, sc.depth, DEFAULT_K, 0.001, device="cpu")
    exp = ref.compute_curvature_profile(sc.mask, sc.depth, DEFAULT_K, 0.001)
    assert got.status == exp.status == "ok"
    assert got.mean_curvature == pytest.approx(exp.mean_curvature, rel=1e-7, abs=1e-9)
    assert got.max_curvature == pytest.approx(exp.max_curvature, rel=1e-7, abs=1e-9)
    a = np.array([[p.x, p.y, p.z] for p in got.spline_points])
    b = np.array([[p.x, p.y, p.z] for p in exp.spline_points])
    assert a.shape == (100, 3) and np.allclose(a, b, atol=1e-9)


def test_early_exits():
    sc = make_scene(0)
    empty = np.zeros_like(sc.mask)
    r = compute_curvature_profile(empty, sc.depth, DEFAULT_K, 0.001, device="cpu")
    assert r.status == "too_few_points" and r.mean_curvature == 0 and r.spline_points == []
    # a tiny blob: >= 100 points but a single x column -> zero bin width -> no edges
    m = np.zeros_like(sc.mask)
    m[100:250, 320] = 1
    r = compute_curvature_profile(m, np.full_like(sc.depth, 500), DEFAULT_K, 0.001, device="cpu")
    assert r.status == "too_few_edge_points" and r.spline_points == []

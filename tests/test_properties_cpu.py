"""Property-based tests (hypothesis) of the CPU-side building blocks over random shapes/data."""
import numpy as np
import torch
import torch.nn.functional as F
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from robotic_discovery_platform_amd.config import GeometryConfig
from robotic_discovery_platform_amd.data.image_io import resize_area, resize_nearest
from robotic_discovery_platform_amd.geometry import reference as gref
from robotic_discovery_platform_amd.geometry.curvature import edges_numpy, sort_edges
from robotic_discovery_platform_amd.parallel.ddp import DistributedShardSampler
from robotic_discovery_platform_amd.proto import vision as pb

SET = settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@SET
@given(h=st.integers(2, 40), w=st.integers(2, 40), fy=st.integers(1, 4), fx=st.integers(1, 4),
       seed=st.integers(0, 2 ** 16))
def test_resize_area_integer_factor_is_block_mean(h, w, fy, fx, seed):
    img = np.random.default_rng(seed).random((h * fy, w * fx, 3))
    got = resize_area(img, (w, h))
    exp = F.avg_pool2d(torch.from_numpy(img).permute(2, 0, 1)[None], (fy, fx))[0].permute(1, 2, 0).numpy()
    assert np.allclose(got, exp, atol=1e-12)


@SET
@given(h=st.integers(1, 50), w=st.integers(1, 50), H=st.integers(1, 80), W=st.integers(1, 80),
       seed=st.integers(0, 2 ** 16))
def test_resize_nearest_matches_floor_mapping(h, w, H, W, seed):
    img = np.random.default_rng(seed).integers(0, 255, (h, w), dtype=np.uint8)
    got = resize_nearest(img, (W, H))
    for y in range(H):
        for x in range(W):
            assert got[y, x] == img[min(int(y * (h / H)), h - 1), min(int(x * (w / W)), w - 1)]


@SET
@given(seed=st.integers(0, 2 ** 16), density=st.floats(0.0, 0.3), zero_frac=st.floats(0.0, 0.5))
def test_edges_match_oracle_on_random_masks(seed, density, zero_frac):
    rng = np.random.default_rng(seed)
    H, W = 48, 64
    mask = (rng.random((H, W)) < density).astype(np.uint8)
    depth = rng.integers(300, 900, (H, W)).astype(np.uint16)
    depth[rng.random((H, W)) < zero_frac] = 0
    K = np.array([[60.0, 0, 32], [0, 60.0, 24], [0, 0, 1]])
    cfg = GeometryConfig()
    e, n = edges_numpy(mask, depth, K, 0.001, cfg)
    pcd = gref.point_cloud(mask, depth, K, 0.001)
    assert n == pcd.shape[0]
    if n < cfg.min_points:
        return
    eo = gref.edge_points(pcd)
    eo = eo[np.argsort(eo[:, 0], kind="stable")]
    assert np.array_equal(sort_edges(e) if len(e) else np.zeros((0, 3)), eo)


@SET
@given(mean=st.floats(-1e3, 1e3), mx=st.floats(-1e3, 1e3), status=st.text(max_size=12),
       mask=st.binary(max_size=64), cov=st.floats(0, 100, width=32),
       pts=st.lists(st.tuples(*[st.floats(-10, 10)] * 3), max_size=5))
def test_proto_roundtrip(mean, mx, status, mask, cov, pts):
    m = pb.AnalysisResponse(mean_curvature=mean, max_curvature=mx, status=status, mask=mask, mask_coverage=cov,
                            spline_points=[pb.Point3D(x=a, y=b, z=c) for a, b, c in pts])
    assert pb.AnalysisResponse.FromString(m.SerializeToString()) == m


@SET
@given(n=st.integers(1, 200), world=st.integers(1, 8), epoch=st.integers(0, 5), drop=st.booleans())
def test_shard_sampler_partitions(n, world, epoch, drop):
    shards = []
    for r in range(world):
        s = DistributedShardSampler(n, r, world, shuffle=True, seed=3, drop_last=drop)
        s.set_epoch(epoch)
        shards.append(list(s))
    assert len({len(x) for x in shards}) == 1  # lockstep: equal length on every rank
    flat = [i for x in shards for i in x]
    if drop:
        assert len(set(flat)) == len(flat)  # disjoint
    else:
        assert set(flat) == set(range(n))  # covers everything (padding repeats)

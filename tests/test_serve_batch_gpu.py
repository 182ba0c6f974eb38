"""Cross-stream batched serving (serve/engine.py BatchEngine, csrc/serve_runtime.cpp BatchRunner) vs the
per-frame pipeline: the same frames give the same masks and curvature whether they run alone (N = 1
graph) or batched with others (N = 2..4 graphs), results come back in each stream's order, and the
encoded (gRPC) path returns the same wire bytes as the single-frame path up to its timing field.
Reference per-frame body: /root/reference/services/vision_analysis/server.py:116-152."""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    from robotic_discovery_platform_amd.serve.bench_serve import prepare_model
    dev = torch.device("cuda")
    model, scenes = prepare_model(dev, train_steps=30, n_scenes=8)
    return model, scenes


def _agree(a, b):
    """mask agreement and curvature closeness of two FrameResults"""
    frac = float((a.mask == b.mask).mean())
    ca, cb = a.curvature, b.curvature
    return frac, ca.status, cb.status, ca.mean_curvature, cb.mean_curvature


@pytest.mark.parametrize("n", [1, 2, 3, 4])
def test_batch_matches_single_frame_pipeline(setup, n):
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K
    from robotic_discovery_platform_amd.serve.engine import SRC_BGR, BatchEngine, FramePipeline
    model, scenes = setup
    single = FramePipeline(model, DEFAULT_K, 0.001, graph=True)
    want = [single.process(sc.color, sc.depth) for sc in scenes[:n]]
    be = BatchEngine(model, DEFAULT_K, 0.001, src=SRC_BGR, positions=4, window_us=200000.0)
    try:
        # hold the launcher until all n frames are staged: they run as ONE batch of n
        pos = [be._acquire() for _ in range(n)]
        tickets = [be.submit(sc.color, sc.depth, pos=p) for sc, p in zip(scenes[:n], pos)]
        got = [be.collect(t) for t in tickets]
        assert be.batch_sizes[n] >= 1, dict(be.batch_sizes)
    finally:
        be.close()
    for a, b in zip(got, want):
        frac, sa, sb, ma, mb = _agree(a, b)
        assert frac > 0.999, frac
        assert sa == sb
        if sa == "ok":
            assert abs(ma - mb) <= 0.05 * abs(mb) + 1e-6, (ma, mb)
        assert abs(a.coverage - b.coverage) < 0.1


def test_pool_sessions_batch_in_order(setup):
    """Four threads with a session each through EnginePool: frames are batched (batch sizes > 1 occur) and
    every session gets its own results back in submission order."""
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K
    from robotic_discovery_platform_amd.serve.engine import EnginePool, FramePipeline
    model, scenes = setup
    single = FramePipeline(model, DEFAULT_K, 0.001, graph=True)
    ref_cov = [single.process(sc.color, sc.depth).coverage for sc in scenes]
    pool = EnginePool(model, DEFAULT_K, 0.001, n=2, graph=True, batch=4)
    errors, seen = [], {}

    def run(k):
        try:
            s = pool.session()
            res = []
            for i in range(40):
                sc = scenes[(i + k) % len(scenes)]
                res += s.submit(sc.color, sc.depth, tag=i)
            res += s.drain()
            seen[k] = res
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    ths = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    [t.start() for t in ths]
    [t.join(timeout=120) for t in ths]
    assert not errors, errors
    for k in range(4):
        tags = [t for t, _ in seen[k]]
        assert tags == list(range(40)), tags
        for i, r in seen[k]:
            assert not isinstance(r, Exception), r
            assert abs(r.coverage - ref_cov[(i + k) % len(scenes)]) < 0.1
    sizes = pool.batchers[0].batch_sizes
    assert sum(c for n, c in sizes.items() if n > 1) > 0, dict(sizes)
    for b in pool.batchers:
        b.close()


def test_batch_encoded_matches_pipeline_wire(setup):
    """The gRPC path's encoded requests: the batched response bytes equal the single-frame path's except
    proc_time_ms (field 7, last in the message)."""
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K
    from robotic_discovery_platform_amd.serve.client import make_request
    from robotic_discovery_platform_amd.serve.engine import SRC_JPEG, BatchEngine, FramePipeline
    model, scenes = setup
    reqs = [make_request(sc.color, sc.depth) for sc in scenes[:3]]
    single = FramePipeline(model, DEFAULT_K, 0.001, graph=True, rgb=True, jpeg=True)
    want = []
    for rq in reqs:
        assert single.submit_encoded(rq.color_image.data, rq.depth_image.data) == 0
        want.append(single.collect_encoded())
    be = BatchEngine(model, DEFAULT_K, 0.001, src=SRC_JPEG, positions=4, window_us=200000.0)
    try:
        pos = [be._acquire() for _ in reqs]
        tick = []
        for rq, p in zip(reqs, pos):
            code, t = be.submit_encoded(rq.color_image.data, rq.depth_image.data, pos=p)
            assert code == 0
            tick.append(t)
        got = [be.collect_encoded(t) for t in tick]
    finally:
        be.close()
    for a, b in zip(got, want):
        # strip field 7 (proc_time_ms: tag 0x3d + 4 bytes) at the end of both
        pa, pb = a.payload, b.payload
        assert pa[-5] == 0x3D and pb[-5] == 0x3D
        if pa[:-5] != pb[:-5]:  # masks may differ in a handful of threshold pixels between batch sizes
            assert abs(a.coverage - b.coverage) < 0.1 and abs(a.mean_curvature - b.mean_curvature) <= \
                0.05 * abs(b.mean_curvature) + 1e-6


def test_batch_all_void_frame_is_skipped_and_reused(setup):
    """A batch whose every position failed staging (undecodable requests) is not launched; its frame goes
    straight back to the rotation and the next batch on it (one frame: the same k, a new generation)
    returns its own results, not a stale launch's."""
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K
    from robotic_discovery_platform_amd.serve.client import make_request
    from robotic_discovery_platform_amd.serve.engine import SRC_JPEG, BatchEngine, FramePipeline
    model, scenes = setup
    single = FramePipeline(model, DEFAULT_K, 0.001, graph=True, rgb=True, jpeg=True)
    reqs = [make_request(sc.color, sc.depth) for sc in scenes[:4]]
    want = []
    for rq in reqs:
        assert single.submit_encoded(rq.color_image.data, rq.depth_image.data) == 0
        want.append(single.collect_encoded())
    be = BatchEngine(model, DEFAULT_K, 0.001, src=SRC_JPEG, frames=1, positions=4, window_us=200000.0)
    try:
        def batch(pairs):
            pos = [be._acquire() for _ in pairs]
            out = [be.submit_encoded(c, d, pos=p) for (c, d), p in zip(pairs, pos)]
            return out
        first = batch([(rq.color_image.data, rq.depth_image.data) for rq in reqs[:2]])
        got_a = [be.collect_encoded(t) for code, t in first if code == 0]
        assert len(got_a) == 2
        # all P positions, so the frame is full: the next acquire waits for the launcher to close it
        # (acquiring several positions before staging any is safe only from a fresh frame)
        void = batch([(b"\xff\xd8not a jpeg", b"junk")] * 4)
        assert all(code != 0 for code, _ in void)
        second = batch([(rq.color_image.data, rq.depth_image.data) for rq in reqs[2:]])
        assert all(code == 0 for code, _ in second)
        got_b = [be.collect_encoded(t) for _, t in second]
        assert sum(be.batch_sizes.values()) == 2, dict(be.batch_sizes)  # the void batch never ran
    finally:
        be.close()
    for a, b in zip(got_a + got_b, want):
        assert abs(a.coverage - b.coverage) < 0.1
        assert abs(a.mean_curvature - b.mean_curvature) <= 0.05 * abs(b.mean_curvature) + 1e-6


@pytest.mark.parametrize("n", [1, 3, 4])
def test_batched_geometry_bitwise_equals_per_frame(setup, n):
    """geo_frames_batch (one launch per stage for n frames, csrc/geometry.hip rdp_geo_edges_batch +
    csrc/geo_spline.hip rdp_geo_spline_batch) on the same model masks and depth frames gives bit-identical
    result vectors and masks as each frame's own GeometryEngine launches."""
    from robotic_discovery_platform_amd.config import GeometryConfig
    from robotic_discovery_platform_amd.data.image_io import resize_nearest
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K
    from robotic_discovery_platform_amd.geometry.curvature import GeometryEngine
    from robotic_discovery_platform_amd.ops import native
    _, scenes = setup
    C = native()
    dev = torch.device("cuda")
    cfg = GeometryConfig()
    H, W = 480, 640
    m256 = [torch.from_numpy(resize_nearest(sc.mask, (256, 256))).to(dev).contiguous() for sc in scenes[:n]]
    m256 = [(m > 0).to(torch.uint8) for m in m256]
    depth = [torch.from_numpy(sc.depth.view(np.int16)).to(dev) for sc in scenes[:n]]
    K = DEFAULT_K
    single = []
    ge = [GeometryEngine(H, W, dev, cfg) for _ in range(n)]
    for j in range(n):
        mask = torch.empty(H, W, dtype=torch.uint8, device=dev)
        mh = torch.zeros(H, W, dtype=torch.uint8).pin_memory()
        ge[j].launch_frame(m256[j], mask, depth[j], K, 0.001, mask_host=mh, host_copy_in_spline=True)
        ge[j].launch_spline(res_out=ge[j].res)
        torch.cuda.synchronize()
        single.append((ge[j].res.cpu().clone(), mask.cpu().clone(), mh.clone()))
    gb = [GeometryEngine(H, W, dev, cfg) for _ in range(n)]
    masks = [torch.empty(H, W, dtype=torch.uint8, device=dev) for _ in range(n)]
    mhs = [torch.zeros(H, W, dtype=torch.uint8).pin_memory() for _ in range(n)]
    C.geo_frames_batch(masks, depth, m256, [g.work_i for g in gb], [g.work_d for g in gb], [g.pts for g in gb],
                       [g.npts for g in gb], [g.out for g in gb], [g.kout for g in gb], [g.cov for g in gb],
                       [g.sorted for g in gb], [g.gperm for g in gb], [g.u for g in gb], [g.res for g in gb], mhs,
                       float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2]), 0.001, cfg.num_bins,
                       cfg.top_k_percent, cfg.min_points, cfg.smoothing, cfg.spline_degree, cfg.num_samples,
                       cfg.deriv_eps, cfg.min_edge_points)
    torch.cuda.synchronize()
    for j in range(n):
        r, m, mh = single[j]
        assert torch.equal(gb[j].res.cpu(), r), j
        assert torch.equal(masks[j].cpu(), m) and torch.equal(mhs[j], mh), j

"""Serving path on the GPU: BN-folded eval conv epilogue, eval U-Net vs the fp32 reference,
preprocess / mask upsample / geometry kernels vs their PyTorch / NumPy references, and the
graph-captured per-frame pipeline vs the reference semantics (server.py:116-152)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C():
    from robotic_discovery_platform_amd.ops import native
    return native()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("N,H,W,C1,C2,Cout", [(2, 16, 16, 64, 0, 64), (1, 9, 13, 64, 64, 128), (1, 8, 8, 256, 256, 256)])
def test_conv_eval_bn_fold_epilogue(C, N, H, W, C1, C2, Cout):
    torch.manual_seed(0)
    dev = "cuda"
    bf = torch.bfloat16
    x1 = torch.randn(N, H, W, C1, device=dev).to(bf)
    x2 = torch.randn(N, H, W, C2, device=dev).to(bf) if C2 else None
    w = (torch.randn(Cout, C1 + C2, 3, 3, device=dev) / math.sqrt(9 * (C1 + C2))).to(bf)
    g, b = torch.rand(Cout, device=dev) + 0.5, torch.randn(Cout, device=dev)
    rm, rv = torch.randn(Cout, device=dev) * 0.1, torch.rand(Cout, device=dev) + 0.5
    coef = torch.zeros(4 * Cout, device=dev)
    C.bn_eval_coef(g, b, rm, rv, 1e-5, coef)
    a = torch.empty(N, H, W, Cout, dtype=bf, device=dev)
    C.conv_fwd(x1, x2, w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous(), 9, 0, a, None, None, 0, coef, 1)
    xin = torch.cat([x1, x2], -1) if C2 else x1
    y = F.conv2d(xin.permute(0, 3, 1, 2).float(), w.float(), padding=1)
    ref = F.relu(F.batch_norm(y, rm, rv, g, b, False, 0.0, 1e-5)).permute(0, 2, 3, 1)
    assert _rel(a, ref) < 1e-2


def test_eval_forward_matches_reference():
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    torch.manual_seed(0)
    dev = torch.device("cuda")
    ref = UNetRef(3, 1).to(dev)
    with torch.no_grad():  # non-trivial running statistics
        for n, b in ref.named_buffers():
            if n.endswith("running_mean"):
                b.normal_(0, 0.1)
            elif n.endswith("running_var"):
                b.uniform_(0.5, 2.0)
    ref.eval()
    nat = UNetNative(3, 1, device=dev, init_from=ref.cpu()).eval()
    ref.to(dev)
    x = torch.rand(2, 3, 128, 128, device=dev)
    xq = x.to(torch.bfloat16).float()
    with torch.no_grad():
        out = nat(x)
        r32 = ref(xq)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            r16 = ref(xq).float()
    e, e16 = _rel(out, r32), _rel(r16, r32)
    print("native", e, "torch-bf16", e16)
    assert e < max(2 * e16, 0.02)


@pytest.mark.parametrize("H,W", [(480, 640), (720, 1280), (256, 256)])
def test_preprocess_matches_torch_antialias(C, H, W):
    from robotic_discovery_platform_amd.serve.engine import aa_tables
    dev = "cuda"
    rng = np.random.default_rng(0)
    bgr = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    ys, yn, yw = aa_tables(H, 256)
    xs, xn, xw = aa_tables(W, 256)
    tabs = [torch.from_numpy(a).to(dev) for a in (ys, yn, yw, xs, xn, xw)]
    out = torch.empty(1, 256, 256, 8, dtype=torch.bfloat16, device=dev)
    C.preprocess(torch.from_numpy(bgr).to(dev), *tabs, out)
    rgb = torch.from_numpy(bgr[..., ::-1].copy()).to(dev).permute(2, 0, 1).float() / 255
    ref = F.interpolate(rgb[None], size=(256, 256), mode="bilinear", align_corners=False, antialias=True)
    got = out[0, :, :, :3].permute(2, 0, 1).float()
    assert (got - ref[0]).abs().max().item() < 1 / 128
    assert out[..., 3:].abs().max().item() == 0


@pytest.mark.parametrize("H,W", [(480, 640), (720, 1280), (100, 333)])
def test_mask_upsample_and_count(C, H, W):
    from robotic_discovery_platform_amd.data.image_io import resize_nearest
    rng = np.random.default_rng(1)
    m = (rng.random((256, 256)) < 0.3).astype(np.uint8)
    out = torch.empty(H, W, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    C.mask_upsample(torch.from_numpy(m).cuda(), out, cnt)
    exp = resize_nearest(m, (W, H))
    assert np.array_equal(out.cpu().numpy(), exp)
    assert int(cnt.item()) == int(exp.sum())


@pytest.mark.parametrize("seed", range(4))
def test_geometry_kernels_match_oracle(seed):
    from robotic_discovery_platform_amd.config import GeometryConfig
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K, make_scene
    from robotic_discovery_platform_amd.geometry import reference as ref
    from robotic_discovery_platform_amd.geometry.curvature import (GeometryEngine, compute_curvature_profile,
                                                                   sort_edges)
    sc = make_scene(seed)
    eng = GeometryEngine(480, 640, torch.device("cuda"), GeometryConfig())
    m = torch.from_numpy(sc.mask).cuda()
    d = torch.from_numpy(sc.depth.view(np.int16)).cuda()
    eng.launch(m, d, DEFAULT_K, 0.001)
    n, E = int(eng.npts.item()), int(eng.hdr.item())
    pcd = ref.point_cloud(sc.mask, sc.depth, DEFAULT_K, 0.001)
    assert n == pcd.shape[0]
    pts = eng.pts[: n * 4].view(n, 4).cpu().numpy()
    assert np.array_equal(pts[:, :3], pcd)  # fp64 deprojection, row-major order
    eo = ref.edge_points(pcd)
    eo = eo[np.argsort(eo[:, 0], kind="stable")]
    got = sort_edges(eng.edges[:E].cpu().numpy())
    assert E == eo.shape[0] and np.array_equal(got, eo)
    # serving form: the select kernel also x-sorts the edge points (fused with the per-bin sort) ==
    # the separate sort launch of the spline stage, bitwise
    m256 = torch.from_numpy(sc.mask[::2, ::2].copy()).cuda()  # any model-resolution mask
    mask_out = torch.empty(480, 640, dtype=torch.uint8, device="cuda")
    eng.launch_frame(m256, mask_out, d, DEFAULT_K, 0.001)
    E2 = int(eng.kout.clamp(max=eng.out.shape[1]).sum().item())
    fused = eng.sorted[:E2].clone()
    c = eng.cfg
    eng.C.geo_spline(eng.out, eng.kout, eng.npts, eng.sorted, eng.gperm, eng.u, eng.res, c.smoothing,
                     c.spline_degree, c.num_samples, c.deriv_eps, c.min_points, c.min_edge_points, eng.cov,
                     presorted=False)
    torch.cuda.synchronize()
    assert E2 > 0 and torch.equal(fused, eng.sorted[:E2])
    r = compute_curvature_profile(sc.mask, sc.depth, DEFAULT_K, 0.001, device="cuda")  # on-device spline
    h = compute_curvature_profile(sc.mask, sc.depth, DEFAULT_K, 0.001, device="cuda", spline="host")
    x = ref.compute_curvature_profile(sc.mask, sc.depth, DEFAULT_K, 0.001)
    for got in (r, h):
        assert got.status == x.status and got.mean_curvature == pytest.approx(x.mean_curvature, rel=1e-7)
        assert got.max_curvature == pytest.approx(x.max_curvature, rel=1e-7)
        assert len(got.spline_points) == len(x.spline_points)
        if x.spline_points:
            a = np.array([[q.x, q.y, q.z] for q in got.spline_points])
            b = np.array([[q.x, q.y, q.z] for q in x.spline_points])
            assert np.abs(a - b).max() < 1e-9
    assert r.n_edge_points == E and r.n_points == n


def test_geometry_large_bins_match_oracle():
    """Every pixel valid (307k points, ~6k per x bin, k ~ 300 > the wave kernel's LDS sort cache):
    the select / sort paths through global memory == the numpy oracle, and the fused serving-form sort ==
    the separate sort launch."""
    from robotic_discovery_platform_amd.config import GeometryConfig
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K
    from robotic_discovery_platform_amd.geometry import reference as ref
    from robotic_discovery_platform_amd.geometry.curvature import GeometryEngine, sort_edges
    rng = np.random.default_rng(5)
    mask = np.ones((480, 640), np.uint8)
    depth = rng.integers(300, 900, (480, 640)).astype(np.uint16)
    eng = GeometryEngine(480, 640, torch.device("cuda"), GeometryConfig())
    d = torch.from_numpy(depth.view(np.int16)).cuda()
    eng.launch(torch.from_numpy(mask).cuda(), d, DEFAULT_K, 0.001)
    E = int(eng.hdr.item())
    pcd = ref.point_cloud(mask, depth, DEFAULT_K, 0.001)
    eo = ref.edge_points(pcd)
    eo = eo[np.argsort(eo[:, 0], kind="stable")]
    got = sort_edges(eng.edges[:E].cpu().numpy())
    assert E == eo.shape[0] and np.array_equal(got, eo)
    assert int(eng.kout.max().item()) > 256
    mask_out = torch.empty(480, 640, dtype=torch.uint8, device="cuda")
    eng.launch_frame(torch.ones(256, 256, dtype=torch.uint8, device="cuda"), mask_out, d, DEFAULT_K, 0.001)
    E2 = int(eng.kout.clamp(max=eng.out.shape[1]).sum().item())
    fused = eng.sorted[:E2].clone()
    c = eng.cfg
    eng.C.geo_spline(eng.out, eng.kout, eng.npts, eng.sorted, eng.gperm, eng.u, eng.res, c.smoothing,
                     c.spline_degree, c.num_samples, c.deriv_eps, c.min_points, c.min_edge_points, eng.cov,
                     presorted=False)
    torch.cuda.synchronize()
    assert E2 == E and torch.equal(fused, eng.sorted[:E2])
    assert np.array_equal(fused.cpu().numpy(), eo[:, :3])


def test_geometry_early_exits():
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K
    from robotic_discovery_platform_amd.geometry.curvature import compute_curvature_profile
    depth = np.full((480, 640), 500, np.uint16)
    r = compute_curvature_profile(np.zeros((480, 640), np.uint8), depth, DEFAULT_K, 0.001, device="cuda")
    assert r.status == "too_few_points"
    m = np.zeros((480, 640), np.uint8)
    m[100:250, 320] = 1
    r = compute_curvature_profile(m, depth, DEFAULT_K, 0.001, device="cuda")
    assert r.status == "too_few_edge_points"


def test_frame_pipeline_matches_reference_semantics():
    from robotic_discovery_platform_amd.data.image_io import resize_nearest
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K, make_scene
    from robotic_discovery_platform_amd.geometry import reference as gref
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.serve.engine import FramePipeline, aa_tables
    torch.manual_seed(0)
    dev = torch.device("cuda")
    nat = UNetNative(3, 1, device=dev).eval()
    # bias the head so the random-init network produces a mask with plenty of pixels
    with torch.no_grad():
        nat.store.view("outc.conv.bias").fill_(0.0)
    sc = make_scene(2)
    pg = FramePipeline(nat, DEFAULT_K, 0.001, graph=True)
    pe = FramePipeline(nat, DEFAULT_K, 0.001, graph=False)
    rg = pg.process(sc.color, sc.depth)
    re_ = pe.process(sc.color, sc.depth)
    assert np.array_equal(rg.mask, re_.mask) and rg.coverage == re_.coverage
    # mask == nearest-upsampled (native logits > 0) of the same preprocessed input. The pipeline's head
    # is fused into the last conv (no activation stored): re-run the executor unfused for the logits.
    ex = pe.ex
    fused256 = pe.m256.view(256, 256).clone()
    ex.forward(head=False, refresh_eval=False)
    head_w = nat.store.view("outc.conv.weight").reshape(-1).float()
    head_b = nat.store.view("outc.conv.bias").float()
    lg = (ex.final.float().reshape(-1, 64) @ head_w + head_b).view(256, 256)
    flip = fused256.bool() != (lg > 0)
    assert (lg[flip].abs() < 1e-3).all()  # only |logit| ~ 0 pixels may differ (dot order)
    m256 = (lg > 0).cpu().numpy().astype(np.uint8)
    exp_full = resize_nearest(m256, (640, 480))
    agree = (exp_full == rg.mask).mean()
    assert agree > 0.999, agree
    assert rg.coverage == pytest.approx(100.0 * rg.mask.sum() / rg.mask.size)
    x = gref.compute_curvature_profile(rg.mask, sc.depth, DEFAULT_K, 0.001)
    assert rg.curvature.status == x.status
    assert rg.curvature.mean_curvature == pytest.approx(x.mean_curvature, rel=1e-7, abs=1e-12)
    # second frame through the graph (buffers reused)
    sc2 = make_scene(5)
    r2 = pg.process(sc2.color, sc2.depth)
    x2 = gref.compute_curvature_profile(r2.mask, sc2.depth, DEFAULT_K, 0.001)
    assert r2.curvature.status == x2.status
    assert r2.curvature.max_curvature == pytest.approx(x2.max_curvature, rel=1e-7, abs=1e-12)


def _jpeg_bytes(rgb, **kw):
    import io
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(rgb, "L" if rgb.ndim == 2 else "RGB").save(buf, format="JPEG", **kw)
    return buf.getvalue()


@pytest.mark.parametrize("H,W", [(480, 640), (37, 53), (1, 9)])
@pytest.mark.parametrize("mode", ["444", "422", "420", "gray"])
def test_jpeg_to_rgb_matches_libjpeg(C, H, W, mode):
    """GPU pixel stage (IDCT + fancy upsampling + YCbCr) == PIL's libjpeg decode, bit for bit."""
    import io
    from PIL import Image
    from robotic_discovery_platform_amd.data.jpeg import coefs_to_rgb_reference, decode_coefs
    rng = np.random.default_rng(H + W)
    y, x = np.mgrid[0:H, 0:W]
    rgb = np.clip(np.stack([x * 4, y * 3, (x + y) * 2], -1) % 256 + rng.integers(-30, 30, (H, W, 3)), 0, 255)
    rgb = rgb.astype(np.uint8)
    if mode == "gray":
        data = _jpeg_bytes(rgb[..., 1].copy(), quality=90)
    else:
        data = _jpeg_bytes(rgb, quality=90, subsampling={"444": 0, "422": 1, "420": 2}[mode], restart_marker_rows=1)
    jc = decode_coefs(data, pin=True)
    assert jc is not None
    dev = torch.device("cuda")
    n = jc.coefs.numel()
    coefs = torch.randint(-2000, 2000, (C.jpeg_max_coefs(H, W),), dtype=torch.int16, device=dev)  # stale tail
    coefs[:n].copy_(jc.coefs)
    meta = jc.meta.to(dev)
    planes = torch.full((C.jpeg_plane_bytes(H, W),), 77, dtype=torch.uint8, device=dev)
    out = torch.zeros(H, W, 3, dtype=torch.uint8, device=dev)
    C.jpeg_to_rgb(coefs, meta[:32], meta[32:], planes, out)
    torch.cuda.synchronize()
    ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    np.testing.assert_array_equal(coefs_to_rgb_reference(jc), ref)


def test_frame_pipeline_jpeg_source_matches_array_source():
    """A JpegCoefs frame through the captured JPEG graph == the same JPEG decoded on the host (RGB)
    through the array graph: same mask, coverage and curvature; one graph serves every sampling."""
    from robotic_discovery_platform_amd.data.image_io import decode_image, encode_jpeg
    from robotic_discovery_platform_amd.data.jpeg import decode_coefs
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K, make_scene
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.serve.engine import SRC_JPEG, FramePipeline
    torch.manual_seed(0)
    nat = UNetNative(3, 1, device=torch.device("cuda")).eval()
    with torch.no_grad():
        nat.store.view("outc.conv.bias").fill_(0.0)
    pj = FramePipeline(nat, DEFAULT_K, 0.001, graph=True, rgb=True, jpeg=True)
    assert SRC_JPEG in pj.graphs  # captured at build, not on the first request
    pe = FramePipeline(nat, DEFAULT_K, 0.001, graph=False)
    for seed, sub in ((2, 2), (5, 0), (7, 1)):
        sc = make_scene(seed)
        data = encode_jpeg(sc.color, 95, restart_rows=1) if sub == 2 else _jpeg_bytes(
            np.ascontiguousarray(sc.color[..., ::-1]), quality=95, subsampling=sub)
        jc = decode_coefs(data, pin=True)
        pj.submit(jc, sc.depth)
        rj = pj.collect()
        arr = decode_image(data, True, "RGB")
        pj.submit(arr, sc.depth, rgb=True)  # host-decoded RGB array through the same pipeline
        ra = pj.collect()
        pe.submit(jc, sc.depth)  # eager program, JPEG source
        rq = pe.collect()
        assert np.array_equal(rj.mask, ra.mask) and rj.coverage == ra.coverage
        assert np.array_equal(rj.mask, rq.mask)
        assert rj.curvature.status == ra.curvature.status
        assert rj.curvature.mean_curvature == ra.curvature.mean_curvature
    with pytest.raises(ValueError):
        small = decode_coefs(encode_jpeg(np.zeros((240, 320, 3), np.uint8)), pin=True)
        pj.submit(small, np.zeros((480, 640), np.uint16))


def test_session_split_submit_and_failed_depth_half():
    """The server's split submission (colour half now, depth half from a future): same result as the
    one-shot submit; a failed depth decode gives that frame an error and leaves the pipeline usable."""
    from concurrent.futures import Future
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K, make_scene
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.serve.engine import EnginePool
    torch.manual_seed(0)
    nat = UNetNative(3, 1, device=torch.device("cuda")).eval()
    with torch.no_grad():
        nat.store.view("outc.conv.bias").fill_(0.0)
    pool = EnginePool(nat, DEFAULT_K, 0.001, n=2, graph=True, rgb=True)
    assert all(p.runner is not None for p in list(pool._pools.values())[0].queue)  # native host path
    sc = make_scene(2)
    rgb = np.ascontiguousarray(sc.color[..., ::-1])
    ref = pool.process(sc.color, sc.depth)

    def fut(v=None, exc=None):
        f = Future()
        f.set_exception(exc) if exc is not None else f.set_result(v)
        return f
    s = pool.session()
    out = []
    out += s.submit(rgb, fut(sc.depth), tag=0, rgb=True)
    out += s.submit(rgb, fut(exc=ValueError("corrupt depth PNG")), tag=1, rgb=True)
    out += s.submit(rgb, fut(sc.depth[:100]), tag=2, rgb=True)  # size mismatch found at the depth half
    out += s.submit(rgb, fut(sc.depth), tag=3, rgb=True)
    out += s.drain()
    res = dict(out)
    assert sorted(res) == [0, 1, 2, 3]
    assert isinstance(res[1], ValueError) and isinstance(res[2], ValueError)
    for k in (0, 3):
        assert np.array_equal(res[k].mask, ref.mask) and res[k].coverage == ref.coverage
        assert res[k].curvature.mean_curvature == ref.curvature.mean_curvature


class _Ctx:
    def set_code(self, c):
        self.code = c

    def set_details(self, d):
        self.details = d


def test_encoded_fast_path_matches_decode_path(tmp_path):
    """The native whole-frame path (request bytes -> pipeline decode, launch, wait, response encode
    without the interpreter lock) answers every frame exactly as the decode path does -- every field
    but proc_time_ms; frames it declines (progressive JPEG, another frame size, 8-bit depth) and corrupt
    ones take the decode path in the same stream, in order."""
    from robotic_discovery_platform_amd.data.image_io import encode_jpeg, encode_png
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K, make_scene
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.proto import vision as pb
    from robotic_discovery_platform_amd.serve.engine import EnginePool
    from robotic_discovery_platform_amd.serve.server import MetricsLog, VisionAnalysisService
    torch.manual_seed(0)
    nat = UNetNative(3, 1, device=torch.device("cuda")).eval()
    with torch.no_grad():
        nat.store.view("outc.conv.bias").fill_(4.0)  # mask ~ everything: fits run on the edge points
    reqs = []
    for seed in (2, 5, 7, 9):
        sc = make_scene(seed)
        reqs.append(pb.AnalysisRequest(color_image=pb.Image(data=encode_jpeg(sc.color, 92, restart_rows=1)),
                                       depth_image=pb.Image(data=encode_png(sc.depth, 1, bands=8))))
    sc = make_scene(3)
    prog = _jpeg_bytes(np.ascontiguousarray(sc.color[..., ::-1]), quality=90, progressive=True)
    reqs.insert(1, pb.AnalysisRequest(color_image=pb.Image(data=prog), depth_image=pb.Image(data=encode_png(sc.depth))))
    small = make_scene(4)
    reqs.insert(3, pb.AnalysisRequest(color_image=pb.Image(data=encode_jpeg(small.color[::2, ::2].copy(), 92)),
                                      depth_image=pb.Image(data=encode_png(small.depth[::2, ::2].copy()))))
    reqs.insert(4, pb.AnalysisRequest(color_image=pb.Image(data=encode_jpeg(sc.color, 92)),
                                      depth_image=pb.Image(data=encode_png((sc.depth // 256).astype(np.uint8)))))
    reqs.append(pb.AnalysisRequest(color_image=pb.Image(data=b"\xff\xd8\xff\xdb"), depth_image=pb.Image(data=b"x")))
    out = {}
    for mode in ("encoded", "decode"):
        pool = EnginePool(nat, DEFAULT_K, 0.001, n=2, graph=True, rgb=True, jpeg=True)
        svc = VisionAnalysisService(pool, MetricsLog(str(tmp_path / f"{mode}.csv")))
        assert svc._encoded
        if mode == "decode":
            svc._encoded = False
        resp = list(svc.AnalyzeActuatorPerformance(iter(reqs), _Ctx()))
        svc.close()
        out[mode] = [pb.AnalysisResponse.FromString(r if isinstance(r, bytes) else r.SerializeToString())
                     for r in resp]
        if mode == "encoded":  # the native path served the plain frames
            assert len(svc.stage_ms["decode_color"]) < len(reqs)
    a, b = out["encoded"], out["decode"]
    assert len(a) == len(b) == len(reqs)
    for x, y in zip(a, b):
        assert x.proc_time_ms > 0 or x.status.startswith("error")
        x.proc_time_ms = y.proc_time_ms = 0.0
        if x.status.startswith("error"):  # the message names a Python object address
            x.status, y.status = x.status.split(" <")[0], y.status.split(" <")[0]
        assert x == y
    assert a[-1].status.startswith("error")
    assert sum(r.status == "ok" and len(r.spline_points) == 100 for r in a) >= 3
    # the metrics log gets the same (mean, max, coverage) rows, timestamps aside
    ra = [r.split(",")[1:] for r in open(tmp_path / "encoded.csv").read().splitlines()[1:]]
    rb = [r.split(",")[1:] for r in open(tmp_path / "decode.csv").read().splitlines()[1:]]
    assert ra == rb and len(ra) == len(reqs) - 1  # the corrupt frame logs no row

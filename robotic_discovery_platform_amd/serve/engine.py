"""Per-frame analysis engine: colour + depth frame -> mask, coverage, curvature profile.

Replaces the serial per-frame body of ``/root/reference/services/vision_analysis/server.py:116-152``
(decode -> ToTensor/Resize(256, antialias) -> UNet -> sigmoid>0.5 -> .cpu() -> cv2 nearest
resize -> numpy/scipy geometry -> coverage) with one device program per frame:

    pinned H2D (colour u8, depth u16)          side HIP stream, async
    preprocess      u8 BGR -> AA resize -> bf16 NHWC8          csrc/serve_kernels.hip
    UNet forward    18 convs (implicit GEMM / row ring), BN folded in the epilogues, eval
                    maxpools fused into the split-K reduces    csrc/conv_igemm.hip, conv_ring.hip
    head mask       1x1 head + (logit > 0) -> u8 256x256, fused into the last conv's epilogue
                    (csrc/conv_ring.hip HEAD; head_mask in csrc/head_loss.hip where it does not apply)
    geo_edges       nearest upsample -> HxW u8 mask + coverage, deproject + compaction + 50-bin
                    top-5 %                                     csrc/geometry.hip
    geo_spline      per-bin x-sort, FITPACK-equivalent spline fit, 100-sample splev + curvature
                                                                csrc/geo_spline.hip
    pinned D2H (mask, 309-double result: curvature, points, coverage, counts)

The device part between the copies is captured once into a hipGraph (torch.cuda.CUDAGraph) and
replayed per frame, so a frame costs one graph launch plus three copies instead of ~90 kernel
launches. ``EnginePool`` holds one ``FramePipeline`` (own executor buffers, stream and graph) per
concurrently served stream; weights are shared and updated in place on hot reload, so graphs stay
valid. ``CpuFramePipeline`` is the same contract on the CPU (plain torch + numpy geometry) for
hosts without a GPU and for the loopback tests.
"""
from __future__ import annotations

import collections
import contextlib
from concurrent import futures
import math
import queue
import threading
import os
import time
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from ..config import GeometryConfig
from ..data.jpeg import JpegCoefs, coefs_to_rgb_reference
from ..geometry.curvature import CurvatureResult, GeometryEngine, compute_curvature_profile
from ..utils import trace

AA_MAXTAP = 16


def aa_tables(n_in: int, n_out: int):
    """torch ``_upsample_bilinear2d_aa`` (align_corners=False) 1-D tables: start[n_out], size[n_out],
    weights[n_out*16] (triangle filter, support = scale when downscaling, normalised)."""
    scale = n_in / n_out
    support = scale if scale >= 1.0 else 1.0
    invscale = 1.0 / scale if scale >= 1.0 else 1.0
    start = np.zeros(n_out, np.int32)
    size = np.zeros(n_out, np.int32)
    w = np.zeros((n_out, AA_MAXTAP), np.float32)
    for i in range(n_out):
        center = scale * (i + 0.5)
        xmin = max(int(center - support + 0.5), 0)
        xsize = min(int(center + support + 0.5), n_in) - xmin
        if xsize > AA_MAXTAP:
            raise ValueError(f"antialias support {xsize} > {AA_MAXTAP} taps (input {n_in} -> {n_out} too large)")
        j = np.arange(xsize)
        ww = np.maximum(0.0, 1.0 - np.abs((j + xmin - center + 0.5) * invscale))
        tot = ww.sum()
        if tot > 0:
            ww = ww / tot
        start[i], size[i] = xmin, xsize
        w[i, :xsize] = ww
    return start, size, w.reshape(-1)


@dataclass
class FrameResult:
    mask: np.ndarray                # HxW uint8 {0,1}
    coverage: float                 # percent of pixels in the mask
    curvature: CurvatureResult
    timings: dict = field(default_factory=dict)
    points: Optional[np.ndarray] = None  # spline points [n, 3] float64 (device fits; the server encodes them)


@dataclass
class WireResult:
    """A frame served end to end natively: its AnalysisResponse wire bytes plus the metrics-log fields."""
    payload: bytes
    mean_curvature: float
    max_curvature: float
    coverage: float
    gpu_ms: float


SRC_BGR, SRC_RGB, SRC_JPEG = 0, 1, 2  # colour sources of a network graph
GEO, GEO_SLOT = "geo", 3  # the geometry graph (FrameRunner slot 3)


def _host_tensor(runner, shape, dtype) -> torch.Tensor:
    """A CPU tensor over fine-grained host memory owned by ``runner`` (kernels write it directly)."""
    import ctypes
    n = int(np.prod(shape)) * np.dtype(dtype).itemsize
    buf = (ctypes.c_uint8 * n).from_address(runner.alloc_host(n))
    return torch.from_numpy(np.frombuffer(buf, dtype=dtype).reshape(shape))


def _stage(dst: torch.Tensor, src: np.ndarray) -> None:
    """Copy a host frame into its pinned staging tensor (on every frame's latency path). A numpy
    assignment: torch's OpenMP-threaded copy was 4x faster alone but its spinning workers cost engine
    and e2e throughput under load, and a worker pool of band copies paid GIL hand-offs
    (profiles/dead_ends.md)."""
    dst.numpy()[...] = src


def _logit(p: float) -> float:
    p = min(max(p, 1e-7), 1 - 1e-7)
    return math.log(p / (1 - p))


# The response mask PNG: deflate level 1 in 8 independent bands (csrc/codecs.cpp; still a standard PNG), encoded
# band-parallel on the host pool after the frame's GPU work -- 8 bands measured 2.4x faster than 4 on the build
# host (0.13 vs 0.31 ms for a 640 x 480 mask, +7 % bytes)
RESP_PNG_LEVEL, RESP_PNG_BANDS = 1, 8


class FramePipeline:
    """One static-shape (H, W) per-frame program on its own HIP stream (GPU, native kernels)."""

    def __init__(self, model, K: np.ndarray, depth_scale: float, H: int = 480, W: int = 640, size: int = 256,
                 threshold: float = 0.5, graph: bool = True, geo_cfg: Optional[GeometryConfig] = None,
                 device: Optional[torch.device] = None, rgb: bool = False, jpeg: bool = False):
        from ..models.unet import UNetNative
        if not isinstance(model, UNetNative):
            raise TypeError("FramePipeline needs the native UNet (UNetNative); use CpuFramePipeline otherwise")
        dev = _norm_device(device if device is not None else model.store.device)
        if dev != _norm_device(model.store.device):
            raise ValueError(f"FramePipeline on {dev} for a model on {model.store.device}: replicate it first")
        # everything below (buffers, stream, graph capture) belongs to the model's GPU, whatever device
        # the calling thread has current
        with torch.cuda.device(dev):
            self._init(model, K, depth_scale, H, W, size, threshold, graph, geo_cfg, dev, rgb, jpeg)

    def _init(self, model, K, depth_scale, H, W, size, threshold, graph, geo_cfg, dev, rgb, jpeg):
        from ..models.unet import UNetExecutor
        from ..ops import native
        self.C = native()
        self.model = model
        self.dev = dev
        self.H, self.W, self.S = H, W, size
        self.K = np.asarray(K, np.float64)
        self.scale = float(depth_scale)
        self.thr_logit = _logit(threshold)
        self.cfg = geo_cfg or GeometryConfig()
        self.stream = torch.cuda.Stream(dev)
        self.ex = UNetExecutor(model, 1, size, size, False, "bce", 1.0)
        # AA resize tables (device)
        ys, yn, yw = aa_tables(H, size)
        xs, xn, xw = aa_tables(W, size)
        self.tab = [torch.from_numpy(a).to(dev) for a in (ys, yn, yw, xs, xn, xw)]
        # device buffers
        self.d_color = torch.empty(H, W, 3, dtype=torch.uint8, device=dev)
        self.d_depth = torch.empty(H, W, dtype=torch.int16, device=dev)
        self.m256 = torch.empty(size * size, dtype=torch.uint8, device=dev)
        self.mask = torch.empty(H, W, dtype=torch.uint8, device=dev)
        ecap = self.cfg.num_bins + int(H * W * self.cfg.top_k_percent) + 1
        self.geo = GeometryEngine(H, W, dev, self.cfg, ecap=ecap)
        # pinned host staging
        self.h_color = torch.empty(H, W, 3, dtype=torch.uint8, pin_memory=True)
        self.h_depth = torch.empty(H, W, dtype=torch.int16, pin_memory=True)
        self.h_mask = torch.empty(H, W, dtype=torch.uint8, pin_memory=True)
        self.h_res = torch.empty(self.geo.res.numel(), dtype=torch.float64, pin_memory=True)
        # JPEG source (data/jpeg.py): entropy-decoded coefficients + geometry / quant tables in, the
        # pixel stage (IDCT, chroma upsampling, YCbCr -> RGB) runs in the frame graph into d_color
        self.d_coef = torch.empty(self.C.jpeg_max_coefs(H, W), dtype=torch.int16, device=dev)
        self.d_meta = torch.zeros(32 + 192, dtype=torch.int32, device=dev)
        self.d_planes = torch.empty(self.C.jpeg_plane_bytes(H, W), dtype=torch.uint8, device=dev)
        self.ev0 = torch.cuda.Event(enable_timing=True)
        self.ev1 = torch.cuda.Event(enable_timing=True)
        self.graphs = {}  # colour source (SRC_BGR / SRC_RGB arrays, SRC_JPEG coefficients) -> hipGraph
        self.use_graph = graph
        self.lock = threading.Lock()
        self._hold = None  # the submitted frame's JPEG buffers, alive until its copies are done
        self._pending_src = None  # colour half submitted, depth half not yet
        # native per-frame host path (csrc/serve_runtime.cpp): staging copies, H2D, graph launch, D2H and
        # events in one call without the GIL; the Python path below stays for eager pipelines
        self.runner = None
        self.zero_copy = False  # the geometry kernels write the mask / result straight to host memory
        if graph and hasattr(self.C, "FrameRunner"):
            r = self.C.FrameRunner(dev.index, self.stream.cuda_stream)
            # mask + result vector in fine-grained host memory the kernels write: no read-back copies
            # after the geometry graph (the copy's launch after a graph cost ~30 us of idle GPU)
            self.h_mask = _host_tensor(r, (H, W), np.uint8)
            self.h_res = _host_tensor(r, (self.geo.res.numel(),), np.float64)
            self.zero_copy = True
            nb = lambda t: t.numel() * t.element_size()  # noqa: E731
            # poll the frame's end event before blocking (FrameRunner.sync_end): a frame is ~0.4 ms of GPU
            # time and a blocking wait's wake-up put 0.05-0.4 ms on the slow frames (profiles/serve_tail.md)
            r.set_spin_us(float(os.environ.get("RDP_SERVE_SPIN_US", "1000")))
            r.set_buffers(self.d_color.data_ptr(), self.h_color.data_ptr(), nb(self.d_color),
                          self.d_depth.data_ptr(), self.h_depth.data_ptr(), nb(self.d_depth),
                          self.d_meta.data_ptr(), nb(self.d_meta), self.d_coef.data_ptr(), nb(self.d_coef),
                          self.mask.data_ptr(), self.h_mask.data_ptr(), 0,
                          self.geo.res.data_ptr(), self.h_res.data_ptr(), 0)
            self.runner = r
        # the graphs for the sources this pipeline will be fed (the gRPC server: JPEG coefficients, or
        # RGB arrays for streams the native decoder does not take) are captured here, at build time --
        # for the configured frame size when the server starts; a pipeline for another frame size is
        # built (and captured) by the first request of that size (EnginePool bounds how many exist)
        if graph:
            self._capture(SRC_RGB if rgb else SRC_BGR)
            if jpeg:
                self._capture(SRC_JPEG)
        else:
            self.refresh_weights()
        # whole encoded requests natively (FrameRunner.submit_encoded): JPEG pipelines with a runner
        self.encoded = bool(graph and jpeg and self.runner is not None)
        if self.encoded:
            self.runner.configure_encoded(H, W, self.cfg.num_samples)

    # ---------------------------------------------------------------- device program
    # A frame is two captured graphs on the pipeline's stream: the network graph of its colour source
    # (JPEG pixel stage, preprocess, U-Net, fused head + threshold -> 256x256 mask) and the geometry
    # graph (mask upsample, back-projection, edge bins, device spline fit). The server enqueues the
    # first as soon as the colour frame is decoded and the second when the depth PNG is, so the network
    # runs while the depth frame is still inflating on the host.
    def _net_program(self, src: int = 0):
        # Measured dead end: the H2D / D2H copies captured INTO the frame graph, depth H2D and mask D2H
        # on a forked branch -- the memcpy nodes replay as blit kernels (20.7 + 17.7 us for colour /
        # depth instead of DMA-engine copies), the fork adds a ~67 us cross-queue gap, and two
        # pipelines no longer overlap: GPU p50 0.622 -> 0.648 ms, pipelined 2307 -> 1502 FPS.
        C, ex, m = self.C, self.ex, self.model
        if src == SRC_JPEG:
            C.jpeg_to_rgb(self.d_coef, self.d_meta[:32], self.d_meta[32:], self.d_planes, self.d_color)
        C.preprocess(self.d_color, *self.tab, ex.x_in, int(src != SRC_BGR))
        # BN-fold coefficients: see refresh_weights(); the head (+ threshold) is fused into the last conv
        ex.forward(head=False, refresh_eval=False,
                   mask_head=(m.store.view("outc.conv.weight").reshape(-1), m.store.view("outc.conv.bias"),
                              self.thr_logit, self.m256))

    def _geo_program(self):
        zc = self.zero_copy
        self.geo.launch_frame(self.m256.view(self.S, self.S), self.mask, self.d_depth, self.K, self.scale,
                              mask_host=self.h_mask if zc else None, host_copy_in_spline=True)
        self.geo.launch_spline(res_out=self.h_res if zc else None)

    def refresh_weights(self):
        """Recompute the BN-fold coefficients from the current weights / running stats (after a
        hot reload). The captured graph reads them -- and every weight layout -- from buffers that a
        reload rewrites in place (``UNetNative.load_state_dict``), so it stays valid."""
        with torch.cuda.device(self.dev), torch.cuda.stream(self.stream):
            self.ex.prepare_eval()
        self.stream.synchronize()

    def wait_idle(self):
        """Block until this pipeline's last submitted frame has left the GPU (its result is dropped)."""
        if self.runner is not None:
            self.runner.abort()  # stream drain: also covers a colour half without its depth half
        else:
            self.stream.synchronize()
        self._hold = None
        self._pending_src = None

    @property
    def graph(self):
        return self.graphs.get(SRC_BGR)

    def _capture_one(self, key, program):
        with torch.cuda.device(self.dev):
            with torch.cuda.stream(self.stream):
                program()  # warm-up (lazy allocations, kernel loading)
            self.stream.synchronize()
            g = torch.cuda.CUDAGraph()
            # thread-local capture: other server threads may use the GPU meanwhile (a late capture of
            # another colour source happens on a live server)
            with torch.cuda.graph(g, stream=self.stream, capture_error_mode="thread_local"):
                program()
        self.graphs[key] = g
        if self.runner is not None:
            self.runner.set_graph(GEO_SLOT if key == GEO else key, g.raw_cuda_graph_exec())

    def _capture(self, src: int):
        if not self.graphs:
            self.refresh_weights()
        self._capture_one(src, lambda: self._net_program(src))
        if GEO not in self.graphs:
            self._capture_one(GEO, self._geo_program)

    # ---------------------------------------------------------------- per frame
    def submit(self, color_bgr, depth: np.ndarray, rgb: bool = False):
        """Stage a frame and enqueue its device work; returns immediately (call ``collect``).
        ``color_bgr``: HxWx3 uint8 array -- OpenCV's BGR, or RGB with ``rgb`` (as the server decodes
        it) -- or a ``JpegCoefs`` (entropy-decoded JPEG; the pixel stage runs in the frame graph)."""
        if depth.shape != (self.H, self.W):
            raise ValueError(f"frame shape {color_bgr.shape}/{depth.shape} != pipeline ({self.H},{self.W})")
        self.submit_color(color_bgr, rgb)
        self.submit_depth(depth)

    def submit_color(self, color, rgb: bool = False):
        """First half of ``submit``: stage the colour frame and enqueue the network graph."""
        if color.shape != (self.H, self.W, 3):
            raise ValueError(f"colour frame {color.shape} != pipeline ({self.H},{self.W})")
        src = SRC_JPEG if isinstance(color, JpegCoefs) else (SRC_RGB if rgb else SRC_BGR)
        if src == SRC_JPEG:
            n = color.coefs.numel()
            if n > self.d_coef.numel() or color.blocks * 64 > n:
                raise ValueError(f"JPEG coefficient planes ({n}) exceed the pipeline's capacity")
        if self.use_graph and src not in self.graphs:  # first frame from this source (stream-ordered)
            self._capture(src)
        with trace.range("serve.frame.enqueue_color"):
            if self.runner is not None:
                if src == SRC_JPEG:
                    self._hold = color  # its (pinned) buffers must outlive the async copies
                    self.runner.submit_jpeg(color.meta.data_ptr(), color.meta.numel() * 4, color.coefs.data_ptr(),
                                            color.coefs.numel() * 2)
                else:
                    self.runner.submit_array(src, np.ascontiguousarray(color))
            else:
                s = self.stream
                if src != SRC_JPEG:
                    _stage(self.h_color, color)
                with torch.cuda.device(self.dev), torch.cuda.stream(s):
                    self.ev0.record(s)
                    if src == SRC_JPEG:
                        self._hold = color
                        self.d_meta.copy_(color.meta, non_blocking=True)
                        self.d_coef[:color.coefs.numel()].copy_(color.coefs, non_blocking=True)
                    else:
                        self.d_color.copy_(self.h_color, non_blocking=True)
                    if self.use_graph:
                        self.graphs[src].replay()
                    else:
                        self._net_program(src)
        self._pending_src = src

    def submit_depth(self, depth: np.ndarray):
        """Second half of ``submit``: stage the depth frame, enqueue the geometry graph and the result
        read-back."""
        if self._pending_src is None:
            raise RuntimeError("submit_depth without submit_color")
        if depth.shape != (self.H, self.W):
            raise ValueError(f"depth frame {depth.shape} != pipeline ({self.H},{self.W})")
        d = depth.view(np.int16) if depth.dtype == np.uint16 else (
            depth if depth.dtype == np.int16 else depth.astype(np.int16))
        with trace.range("serve.frame.enqueue_depth"):
            if self.runner is not None:
                self.runner.submit_depth(np.ascontiguousarray(d))
            else:
                s = self.stream
                _stage(self.h_depth, d)
                with torch.cuda.device(self.dev), torch.cuda.stream(s):
                    self.d_depth.copy_(self.h_depth, non_blocking=True)
                    if self.use_graph:
                        self.graphs[GEO].replay()
                    else:
                        self._geo_program()
                    if not self.zero_copy:
                        self.h_mask.copy_(self.mask, non_blocking=True)
                        self.h_res.copy_(self.geo.res, non_blocking=True)
                    self.ev1.record(s)
        self._pending_src = None

    def submit_encoded(self, color: bytes, depth: bytes) -> int:
        """A request's colour JPEG + 16-bit depth PNG bytes, decoded and launched natively without the
        interpreter lock (csrc/serve_runtime.cpp). 0: in flight (``collect_encoded``); 1 / 2: not a
        frame this path takes (other JPEG kinds, other sizes, 8-bit depth), 3: corrupt -- nothing in
        flight, the caller decodes it itself."""
        if not self.encoded:
            return 1
        with trace.range("serve.frame.submit_encoded"):
            return self.runner.submit_encoded(color, depth)

    def submit_request(self, raw: bytes) -> int:
        """A whole serialized AnalysisRequest, its image payloads read in place natively
        (csrc/serve_runtime.cpp parse_request); codes as ``submit_encoded`` (1 also for a message the native
        parser does not take)."""
        if not self.encoded:
            return 1
        with trace.range("serve.frame.submit_request"):
            return self.runner.submit_request(raw)

    def collect_encoded(self):
        """WireResult of the frame ``submit_encoded`` launched, or a FrameResult when its spline fit
        must finish on the host (the device's capacity was exceeded: rare)."""
        with trace.range("serve.frame.collect_encoded"):
            payload, mean, maxc, cov, st, gpu_ms = self.runner.collect_encoded(RESP_PNG_LEVEL, RESP_PNG_BANDS)
        if st == 4:
            from ..geometry.curvature import coverage_from_device
            h_res = self.h_res.numpy()
            res = self.geo.finish_device(h_res)
            cov = 100.0 * coverage_from_device(h_res, self.cfg) / (self.H * self.W)
            return FrameResult(self.h_mask.numpy().copy(), cov, res, {"gpu_ms": gpu_ms})
        return WireResult(payload, mean, maxc, cov, gpu_ms)

    def abort(self):
        """Drop a frame whose depth half will not come (its decode failed)."""
        self.wait_idle()

    def collect(self) -> FrameResult:
        t0 = time.perf_counter()
        with trace.range("serve.frame.wait_gpu"):
            if self.runner is not None:
                gpu_ms = self.runner.wait()
            else:
                self.ev1.synchronize()
                gpu_ms = self.ev0.elapsed_time(self.ev1)
            self._hold = None
        t1 = time.perf_counter()
        from ..geometry.curvature import coverage_from_device
        h_res = self.h_res.numpy()
        count = coverage_from_device(h_res, self.cfg)
        with trace.range("serve.frame.spline_fit"):  # device result -> CurvatureResult (host fit only as fallback)
            res = self.geo.finish_device(h_res)
        pts = None
        if int(h_res[0]) == 0 and res.status == "ok":  # fitted on the device: the points are in the result
            pts = h_res[8:8 + 3 * self.cfg.num_samples].reshape(-1, 3).copy()
        t2 = time.perf_counter()
        cov = 100.0 * count / (self.H * self.W)
        # gpu_ms: colour-half start -> results on the host (includes any wait for the depth half)
        return FrameResult(self.h_mask.numpy().copy(), cov, res,
                           {"gpu_ms": gpu_ms, "wait_ms": (t1 - t0) * 1e3, "fit_ms": (t2 - t1) * 1e3}, pts)

    def process(self, color_bgr: np.ndarray, depth: np.ndarray) -> FrameResult:
        with self.lock:
            self.submit(color_bgr, depth)
            return self.collect()


class BatchEngine:
    """Frames of several client streams run as ONE batched device program (one replica, one GPU).

    The network is latency-bound at N = 1 (0.379 ms; 0.476 at N = 2, 0.700 at N = 4), and N = 1 graphs of
    concurrent streams time-slice the GPU instead of sharing its width: four streams served 3,179 frames/s
    against 3,410 for one (driver, round 5). Here a frame takes a position j of the open batch frame k
    (K frames rotate, P positions each), is decoded / staged straight into that position's pinned buffers
    (natively, no interpreter lock: csrc/serve_runtime.cpp BatchRunner), and a launcher thread closes the
    batch and launches it as one captured graph -- per position the JPEG pixel stage and preprocess into
    slice j of the batch-n input, the U-Net at batch n with the head + threshold fused, then per position
    the geometry (mask upsample, back-projection, edge bins, spline fit) writing that position's host
    result memory. Launch policy: at once when the batch is full or the GPU has nothing of this engine in
    flight; otherwise the batch keeps filling until the GPU drains or ``window_us`` passed since its first
    frame -- under load batches grow, when idle a frame never waits.

    Reference per-frame body: ``/root/reference/services/vision_analysis/server.py:116-152`` (10 worker
    threads sharing one model, ``:172``)."""

    def __init__(self, model, K, depth_scale, H: int = 480, W: int = 640, size: int = 256, threshold: float = 0.5,
                 geo_cfg: Optional[GeometryConfig] = None, device: Optional[torch.device] = None, src: int = SRC_JPEG,
                 frames: Optional[int] = None, positions: int = 4, window_us: float = 300.0,
                 lanes: Optional[int] = None):
        dev = _norm_device(device if device is not None else model.store.device)
        if lanes is None:
            lanes = int(os.environ.get("RDP_BATCH_LANES", "1"))
        lanes = max(1, int(lanes))
        if frames is None:  # per lane: one running, one queued, one filling, one being collected
            frames = 4 * lanes
        with torch.cuda.device(dev):
            self._init(model, K, depth_scale, H, W, size, threshold, geo_cfg, dev, src, max(frames, lanes), positions,
                       window_us, lanes)

    def _init(self, model, K, depth_scale, H, W, size, threshold, geo_cfg, dev, src, frames, positions, window_us,
              lanes):
        from ..models.unet import UNetExecutor
        from ..ops import native
        C = self.C = native()
        self.model, self.dev, self.src = model, dev, src
        self.H, self.W, self.S = H, W, size
        self.K = np.asarray(K, np.float64)
        self.scale = float(depth_scale)
        self.thr_logit = _logit(threshold)
        self.cfg = geo_cfg or GeometryConfig()
        self.nf, self.P = int(frames), int(positions)
        self.window = window_us * 1e-6
        self.max_wait = float(os.environ.get("RDP_BATCH_MAX_WAIT_US", "2000")) * 1e-6
        # lanes: batch frame k runs on lane k % lanes (its own stream and executor activations), so two
        # batches can be on the GPU at once -- concurrent streams overlap one batch's latency-bound stages
        # with the other's work, as concurrent N = 1 graphs do
        self.lanes = lanes
        self.lane_stream = [torch.cuda.Stream(dev) for _ in range(lanes)]
        self.stream = self.lane_stream[0]
        ys, yn, yw = aa_tables(H, size)
        xs, xn, xw = aa_tables(W, size)
        self.tab = [torch.from_numpy(a).to(dev) for a in (ys, yn, yw, xs, xn, xw)]
        jpeg = src == SRC_JPEG
        coef_cap = C.jpeg_max_coefs(H, W) if jpeg else 0
        ecap = self.cfg.num_bins + int(H * W * self.cfg.top_k_percent) + 1
        self.geo = [[GeometryEngine(H, W, dev, self.cfg, ecap=ecap) for _ in range(self.P)] for _ in range(self.nf)]
        self.masks = [[torch.empty(H, W, dtype=torch.uint8, device=dev) for _ in range(self.P)] for _ in range(self.nf)]
        res_len = self.geo[0][0].res.numel()
        self.runner = C.BatchRunner(dev.index, self.stream.cuda_stream, self.nf, self.P, H, W, self.cfg.num_samples,
                                    src, coef_cap * 2, res_len)
        self.runner.set_spin_us(float(os.environ.get("RDP_SERVE_SPIN_US", "1000")))
        for k in range(self.nf):
            self.runner.set_frame_stream(k, self.lane_stream[k % lanes].cuda_stream)
        # inputs of (batch frame k, position j) on the device: frame k + 1's uploads (copy engine, copy
        # stream) run while frame k computes; the JPEG pixel stage's planes / colour are per position
        nk, P = self.nf, self.P
        up_u8 = (lambda: torch.empty(H, W, 3, dtype=torch.uint8, device=dev))  # noqa: E731
        self.d_depth = [[torch.empty(H, W, dtype=torch.int16, device=dev) for _ in range(P)] for _ in range(nk)]
        if jpeg:
            self.d_coef = [[torch.empty(coef_cap, dtype=torch.int16, device=dev) for _ in range(P)] for _ in range(nk)]
            self.d_meta = [[torch.zeros(32 + 192, dtype=torch.int32, device=dev) for _ in range(P)] for _ in range(nk)]
            self.d_planes = [torch.empty(C.jpeg_plane_bytes(H, W), dtype=torch.uint8, device=dev) for _ in range(P)]
            col = [up_u8() for _ in range(P)]
            self.d_color = [col for _ in range(nk)]
        else:
            self.d_color = [[up_u8() for _ in range(P)] for _ in range(nk)]
        for k in range(nk):
            for j in range(P):
                up = self.d_coef[k][j] if jpeg else self.d_color[k][j]
                self.runner.set_device(k, j, up.data_ptr(), self.d_meta[k][j].data_ptr() if jpeg else 0,
                                       self.d_depth[k][j].data_ptr())
        # the per-frame stages of a batch (JPEG pixel stage + preprocess, geometry) run as parallel branches
        # of its graph, each frame's on a capture stream of its own
        self.branch = [torch.cuda.Stream(dev) for _ in range(P)]
        # host results of (k, j): mask + result vector in the runner's fine-grained host memory
        def host(kind, k, j, shape, dtype):
            import ctypes
            n = int(np.prod(shape)) * np.dtype(dtype).itemsize
            buf = (ctypes.c_uint8 * n).from_address(self.runner.host_ptr(kind, k, j))
            return torch.from_numpy(np.frombuffer(buf, dtype=dtype).reshape(shape))
        self.h_mask = [[host(3, k, j, (H, W), np.uint8) for j in range(self.P)] for k in range(self.nf)]
        self.h_res = [[host(4, k, j, (res_len,), np.float64) for j in range(self.P)] for k in range(self.nf)]
        # one eval executor per (lane, batch size): activations shared by the batch frames of a lane (one stream)
        self.exl = [{n: UNetExecutor(model, n, size, size, False, "bce", 1.0) for n in range(1, self.P + 1)}
                    for _ in range(lanes)]
        self.m256l = [{n: torch.empty(n * size * size, dtype=torch.uint8, device=dev) for n in range(1, self.P + 1)}
                      for _ in range(lanes)]
        self.ex, self.m256 = self.exl[0], self.m256l[0]
        self.graphs = {}
        self.refresh_weights()
        for k in range(self.nf):
            for n in range(1, self.P + 1):
                self._capture(k, n)
        self._init_batching()

    def _init_batching(self):
        """Batching state, guarded by one lock with three conditions: the launcher waits on ``_cv`` (a
        frame staged), collectors on ``_cv_launched`` (a batch launched), acquirers and ``hold`` on
        ``_cv_free`` (a frame closed or freed) -- each event wakes only the threads that wait for it, not
        every session thread of the replica (``RDP_BATCH_ONECV=1``: one condition for all, A/B)."""
        self._lock = threading.Lock()
        self._cv = threading.Condition(self._lock)
        if os.environ.get("RDP_BATCH_ONECV", "0") == "1":
            self._cv_launched = self._cv_free = self._cv
        else:
            self._cv_launched = threading.Condition(self._lock)
            self._cv_free = threading.Condition(self._lock)
        self._free = collections.deque(range(self.nf))
        self._open = None        # batch frame taking new frames
        self._acq = 0            # positions handed out in the open frame
        self._ready = 0          # of those, staged
        self._void = set()       # positions of the open frame whose staging failed (run, result dropped)
        self._t_first = 0.0
        self._refs = [0] * self.nf  # results of a launched frame not yet collected
        self._gen = [0] * self.nf  # times each frame was opened
        self._launched_gen = [0] * self.nf  # ... and launched (a collect waits for its frame's launch)
        self._launched = collections.deque()  # launched frames, oldest first (GPU occupancy)
        self._done_evs = {}
        self.batch_sizes = collections.Counter()
        # callable -> how many client streams feed this engine now (EnginePool: sessions active in the last
        # few ms), the batch size to wait for; None: launch as the GPU frees up
        self.target = getattr(self, "target", None)
        self._stop = False
        self._error = None       # what ended the launcher, if a launch raised
        self._th = threading.Thread(target=self._launcher, name="rdp-batch-launcher", daemon=True)
        self._th.start()

    # ------------------------------------------------------------------ device program
    def _fork(self, n: int, body):
        """Run ``body(j)`` for j < n, frame j's work on branch stream j (forked from and joined back into the
        current stream: parallel branches of a captured graph) with ``RDP_BATCH_BRANCHES=1``; by default in
        order (the branches measured 0.06 ms slower per 4-frame batch: profiles/serve_batch.md)."""
        if n == 1 or os.environ.get("RDP_BATCH_BRANCHES", "0") == "0":
            for j in range(n):
                body(j)
            return
        main = torch.cuda.current_stream()
        for j in range(n):
            b = self.branch[j]
            b.wait_stream(main)
            with torch.cuda.stream(b):
                body(j)
        for j in range(n):
            main.wait_stream(self.branch[j])

    def _program(self, k: int, n: int):
        C, m = self.C, self.model
        lane = k % self.lanes
        ex = self.exl[lane][n]
        m256 = self.m256l[lane][n]

        def pre(j):
            if self.src == SRC_JPEG:
                C.jpeg_to_rgb(self.d_coef[k][j], self.d_meta[k][j][:32], self.d_meta[k][j][32:], self.d_planes[j],
                              self.d_color[k][j])
            C.preprocess(self.d_color[k][j], *self.tab, ex.x_in[j:j + 1], int(self.src != SRC_BGR))

        if os.environ.get("RDP_BATCH_PRE", "1") != "0":
            # every frame's JPEG pixel stage (2 launches) and preprocess (1 launch), blockIdx.y = frame
            jp = self.src == SRC_JPEG
            C.batch_preprocess([self.d_coef[k][j] for j in range(n)] if jp else [],
                               [self.d_meta[k][j] for j in range(n)] if jp else [],
                               [self.d_planes[j] for j in range(n)] if jp else [],
                               [self.d_color[k][j] for j in range(n)], *self.tab, ex.x_in, int(self.src != SRC_BGR))
        else:
            self._fork(n, pre)
        ex.forward(head=False, refresh_eval=False,
                   mask_head=(m.store.view("outc.conv.weight").reshape(-1), m.store.view("outc.conv.bias"),
                              self.thr_logit, m256))
        S2 = self.S * self.S

        if os.environ.get("RDP_BATCH_GEO", "1") != "0":
            # every frame's geometry in one launch per stage (csrc/geometry.hip / geo_spline.hip batch forms)
            gs = [self.geo[k][j] for j in range(n)]
            c, Kc = self.cfg, self.K
            C.geo_frames_batch([self.masks[k][j] for j in range(n)], [self.d_depth[k][j] for j in range(n)],
                               [m256[j * S2:(j + 1) * S2].view(self.S, self.S) for j in range(n)],
                               [g.work_i for g in gs], [g.work_d for g in gs], [g.pts for g in gs],
                               [g.npts for g in gs], [g.out for g in gs], [g.kout for g in gs], [g.cov for g in gs],
                               [g.sorted for g in gs], [g.gperm for g in gs], [g.u for g in gs],
                               [self.h_res[k][j] for j in range(n)], [self.h_mask[k][j] for j in range(n)],
                               float(Kc[0, 0]), float(Kc[1, 1]), float(Kc[0, 2]), float(Kc[1, 2]), self.scale,
                               c.num_bins, c.top_k_percent, c.min_points, c.smoothing, c.spline_degree,
                               c.num_samples, c.deriv_eps, c.min_edge_points)
            return

        def geo(j):
            g = self.geo[k][j]
            g.launch_frame(m256[j * S2:(j + 1) * S2].view(self.S, self.S), self.masks[k][j],
                           self.d_depth[k][j], self.K, self.scale, mask_host=self.h_mask[k][j], host_copy_in_spline=True)
            g.launch_spline(res_out=self.h_res[k][j])

        self._fork(n, geo)

    def _capture(self, k: int, n: int):
        st = self.lane_stream[k % self.lanes]
        with torch.cuda.device(self.dev):
            with torch.cuda.stream(st):
                self._program(k, n)  # warm-up (lazy allocations, kernel loading)
            st.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st, capture_error_mode="thread_local"):
                self._program(k, n)
        self.graphs[(k, n)] = g
        self.runner.set_graph(k, n, g.raw_cuda_graph_exec())

    def refresh_weights(self):
        """BN-fold coefficients (and fragment-major eval weights) of every batch executor from the current
        weights; the graphs read them from buffers rewritten in place."""
        with torch.cuda.device(self.dev), torch.cuda.stream(self.stream):
            for exs in self.exl:
                for ex in exs.values():
                    ex.prepare_eval()
        self.stream.synchronize()

    def wait_idle(self):
        self.runner.drain()

    # ------------------------------------------------------------------ batching
    def _acquire(self, block: bool = True):
        """(k, j, generation) of a position in the open batch frame; None if ``block`` is False and none is
        free."""
        with self._cv:
            while True:
                if self._stop:
                    raise RuntimeError("BatchEngine closed" if self._error is None
                                       else f"BatchEngine launch failed: {self._error!r}")
                if self._open is None and self._free:
                    self._open = self._free.popleft()
                    self._acq = self._ready = 0
                    self._void = set()
                    self._gen[self._open] += 1
                if self._open is not None and self._acq < self.P:
                    j = self._acq
                    self._acq += 1
                    return self._open, j, self._gen[self._open]
                if not block:
                    return None
                self._cv_free.wait()

    def _staged(self, k: int, j: int, ok: bool):
        with self._cv:
            if not ok:
                self._void.add(j)
            if self._ready == 0:
                self._t_first = time.perf_counter()
            self._ready += 1
            self._cv.notify_all()

    def _gpu_pending(self) -> int:
        """Launched frames whose device work has not finished (polled, no blocking)."""
        while self._launched and self._done(self._launched[0]):
            self._launched.popleft()
        return len(self._launched)

    def _done(self, k: int) -> bool:
        ev = self._done_evs.get(k)
        return ev is None or ev.query()

    def _launcher(self):
        with torch.cuda.device(self.dev):
            while True:
                with self._cv:
                    while True:
                        if self._stop:
                            return
                        k, acq, ready = self._open, self._acq, self._ready
                        if k is not None and ready > 0 and ready == acq:
                            # every active stream's frame is in (each stream has one frame waiting at a time
                            # in steady state), or the batch is full, or the window since its first frame
                            # passed; with no stream count (target None) a lone batch also goes when the GPU
                            # has nothing of this engine in flight
                            tgt = self.target() if self.target is not None else None
                            waited = time.perf_counter() - self._t_first
                            if tgt is None:  # no stream count: launch as a lane frees up
                                go = acq >= self.P or self._gpu_pending() < self.lanes or waited >= self.window
                            else:
                                # a partial batch goes early only onto an idle GPU (after the window) or after
                                # max_wait: while a batch runs, launching would only queue it behind -- it
                                # keeps filling instead (frames of a stream that was preempted still join)
                                go = (acq >= min(self.P, max(tgt, 1)) or
                                      (waited >= self.window and self._gpu_pending() < self.lanes) or
                                      waited >= self.max_wait)
                            if go:
                                break
                            # sleep until the window ends (a new frame notifies earlier), then poll the GPU
                            # every 100 us: a short fixed poll woke this thread ~20k times a second, each
                            # wake-up taking the interpreter lock from the stream threads
                            t = self.window - waited if waited < self.window else 100e-6
                            self._cv.wait(timeout=max(20e-6, min(t, self.max_wait - waited)))
                            continue
                        self._cv.wait(timeout=1e-3 if k is not None and ready > 0 else None)
                    n, void = acq, self._void
                    gen = self._gen[k]  # k may be reopened (a new generation) as soon as it is freed
                    self._open = None  # the next acquire opens a new frame
                    self._refs[k] = n - len(void)
                    if self._refs[k] == 0:  # every position failed staging: nothing to run or collect
                        self._free.append(k)
                    self._cv_free.notify_all()  # the next acquire opens a frame
                    if self._refs[k] == 0:
                        continue
                try:
                    self.runner.launch(k, n)  # uploads + graph + end event (no GIL)
                    ev = self._done_evs.get(k)
                    if ev is None:
                        ev = self._done_evs[k] = torch.cuda.Event()
                    ev.record(self.lane_stream[k % self.lanes])
                except BaseException as e:  # collectors must not wait for a launch that never comes
                    with self._cv:
                        self._error = e
                        self._stop = True
                        self._notify_every()
                    return
                with self._cv:
                    self._launched.append(k)
                    self._launched_gen[k] = gen
                    self.batch_sizes[n] += 1
                    self._cv_launched.notify_all()

    def _await_launch(self, k: int, gen: int):
        with self._cv:
            while self._launched_gen[k] != gen:
                if self._stop:
                    raise RuntimeError("BatchEngine closed" if self._error is None
                                       else f"BatchEngine launch failed: {self._error!r}") from self._error
                self._cv_launched.wait()

    def _release(self, k: int):
        with self._cv:
            self._refs[k] -= 1
            if self._refs[k] == 0:
                self._free.append(k)
                self._cv_free.notify_all()

    def submit_encoded(self, color: bytes, depth: bytes, pos=None):
        """(code, ticket): 0 and the frame's (k, j) when it is staged for the next batch; otherwise nothing
        of it runs (1 / 2 / 3 as FramePipeline.submit_encoded: the caller decodes it itself). ``pos``: a
        position already taken with ``_acquire``."""
        k, j, gen = pos if pos is not None else self._acquire()
        try:
            code = self.runner.decode(k, j, color, depth)
        except BaseException:
            self._staged(k, j, False)
            raise
        self._staged(k, j, code == 0)
        return code, (k, j, gen)

    def submit_request(self, raw: bytes, pos=None):
        """``submit_encoded`` from a whole serialized AnalysisRequest (payloads read in place natively)."""
        k, j, gen = pos if pos is not None else self._acquire()
        try:
            code = self.runner.decode_request(k, j, raw)
        except BaseException:
            self._staged(k, j, False)
            raise
        self._staged(k, j, code == 0)
        return code, (k, j, gen)

    def submit(self, color, depth: np.ndarray, pos=None):
        """An HxWx3 u8 colour array (this engine's channel order) + HxW depth frame; returns the ticket."""
        if self.src == SRC_JPEG:
            raise ValueError("BatchEngine(src=JPEG) takes encoded requests")
        d = depth.view(np.int16) if depth.dtype == np.uint16 else depth
        k, j, gen = pos if pos is not None else self._acquire()
        try:
            self.runner.stage(k, j, np.ascontiguousarray(color), np.ascontiguousarray(d))
        except BaseException:
            self._staged(k, j, False)
            raise
        self._staged(k, j, True)
        return k, j, gen

    def collect_encoded(self, ticket):
        k, j, gen = ticket
        try:
            self._await_launch(k, gen)
            payload, mean, maxc, cov, st, gpu_ms = self.runner.collect_encoded(k, j, RESP_PNG_LEVEL, RESP_PNG_BANDS)
            if st == 4:  # the fit needs the host (device capacity exceeded): from this position's edge buffers
                r = self._frame_result(k, j, gpu_ms)
                return r
            return WireResult(payload, mean, maxc, cov, gpu_ms)
        finally:
            self._release(k)

    def collect(self, ticket) -> FrameResult:
        k, j, gen = ticket
        try:
            self._await_launch(k, gen)
            gpu_ms = self.runner.wait(k)
            return self._frame_result(k, j, gpu_ms)
        finally:
            self._release(k)

    def _frame_result(self, k, j, gpu_ms) -> FrameResult:
        from ..geometry.curvature import coverage_from_device
        h_res = self.h_res[k][j].numpy()
        count = coverage_from_device(h_res, self.cfg)
        with torch.cuda.device(self.dev):
            res = self.geo[k][j].finish_device(h_res)
        pts = None
        if int(h_res[0]) == 0 and res.status == "ok":
            pts = h_res[8:8 + 3 * self.cfg.num_samples].reshape(-1, 3).copy()
        return FrameResult(self.h_mask[k][j].numpy().copy(), 100.0 * count / (self.H * self.W), res,
                           {"gpu_ms": gpu_ms}, pts)

    def hold(self):
        """Take every batch frame (waits until each is free: nothing in flight or uncollected), so the
        weights can be swapped; ``unhold`` gives them back."""
        got = []
        with self._cv:
            while len(got) < self.nf:
                if self._open is not None and self._acq == 0:  # an open frame nobody took a position in
                    self._free.append(self._open)
                    self._open = None
                if self._free:
                    got.append(self._free.popleft())
                    continue
                if self._stop:  # the launcher is gone: a half-filled frame would never free
                    self._free.extend(got)
                    raise RuntimeError("BatchEngine closed")
                self._cv_free.wait()
        self._held = got
        self.runner.drain()

    def unhold(self):
        with self._cv:
            self._free.extend(getattr(self, "_held", []))
            self._held = []
            self._cv_free.notify_all()

    def close(self):
        with self._cv:
            self._stop = True
            self._notify_every()
        self._th.join(timeout=5.0)

    def _notify_every(self):  # (lock held) stop / failure: wake every waiter
        self._cv.notify_all()
        self._cv_launched.notify_all()
        self._cv_free.notify_all()
        self.runner.drain()


class CpuFramePipeline:
    """Same contract on the CPU: torch (any UNet module) + numpy geometry + native C++ spline."""

    def __init__(self, model, K, depth_scale, H: int = 480, W: int = 640, size: int = 256, threshold: float = 0.5,
                 geo_cfg: Optional[GeometryConfig] = None, **_):
        self.model, self.K, self.scale = model, np.asarray(K, np.float64), float(depth_scale)
        self.H, self.W, self.S, self.thr = H, W, size, threshold
        self.cfg = geo_cfg or GeometryConfig()
        self.lock = threading.Lock()
        self._pending = None

    def refresh_weights(self):
        pass  # the torch module reads its parameters directly

    def wait_idle(self):
        self._pending = None

    def submit(self, color_bgr, depth: np.ndarray, rgb: bool = False):
        if color_bgr.shape != (self.H, self.W, 3) or depth.shape != (self.H, self.W):
            raise ValueError(f"frame shape {color_bgr.shape}/{depth.shape} != pipeline ({self.H},{self.W})")
        if isinstance(color_bgr, JpegCoefs):  # (the server only sends these to GPU pipelines)
            color_bgr, rgb = coefs_to_rgb_reference(color_bgr), True
        self._pending = (color_bgr[..., ::-1] if rgb else color_bgr, depth)

    def submit_color(self, color, rgb: bool = False):
        if color.shape != (self.H, self.W, 3):
            raise ValueError(f"colour frame {color.shape} != pipeline ({self.H},{self.W})")
        self._color = (color, rgb)

    def submit_depth(self, depth: np.ndarray):
        color, rgb = self._color
        self._color = None
        self.submit(color, depth, rgb)

    def abort(self):
        self._color = self._pending = None

    def collect(self) -> FrameResult:
        color_bgr, depth = self._pending
        self._pending = None
        return self.process(color_bgr, depth)

    def process(self, color_bgr: np.ndarray, depth: np.ndarray) -> FrameResult:
        import torch.nn.functional as F
        from ..data.image_io import resize_nearest
        t0 = time.perf_counter()
        rgb = torch.from_numpy(np.ascontiguousarray(color_bgr[..., ::-1])).permute(2, 0, 1).float().div(255)
        x = F.interpolate(rgb[None], size=(self.S, self.S), mode="bilinear", align_corners=False, antialias=True)
        with torch.no_grad():
            out = self.model(x.to(next(self.model.parameters()).device))
        m = (torch.sigmoid(out.float()) > self.thr)[0, 0].cpu().numpy().astype(np.uint8)
        mask = resize_nearest(m, (color_bgr.shape[1], color_bgr.shape[0]))
        t1 = time.perf_counter()
        res = compute_curvature_profile(mask, depth, self.K, self.scale, self.cfg, device="cpu")
        cov = 100.0 * np.count_nonzero(mask) / mask.size
        return FrameResult(mask, cov, res, {"model_ms": (t1 - t0) * 1e3,
                                             "fit_ms": (time.perf_counter() - t1) * 1e3})


def _norm_device(device) -> torch.device:
    """``cuda`` without an index -> ``cuda:<current>`` (so equal devices compare equal)."""
    device = torch.device(device)
    if device.type == "cuda" and device.index is None:
        return torch.device("cuda", torch.cuda.current_device())
    return device


def _on(device):
    """``torch.cuda.device(device)`` for a GPU device, else a no-op context."""
    device = torch.device(device)
    return torch.cuda.device(device) if device.type == "cuda" else contextlib.nullcontext()


def replicate_model(model, device: torch.device):
    """A copy of ``model`` on ``device`` (same architecture, weights and BN statistics); built with
    ``device`` current, so every launch of its construction (bf16 shadow, weight re-layouts) runs on
    that GPU."""
    if _is_native(model):
        from ..models.unet import UNetNative
        with _on(device):
            rep = UNetNative(model.n_channels, model.n_classes, bilinear=model.bilinear, base_width=model.base_width,
                             depth=model.depth, device=torch.device(device))
            rep.load_state_dict({k: v.detach() for k, v in model.state_dict().items()})
        return rep.eval()
    import copy
    return copy.deepcopy(model).to(device).eval()


class EnginePool:
    """Per-frame pipelines for the server's streams, with one model replica per GPU.

    * ``devices`` (SURVEY.md §2.4 serving concurrency): one replica of the weights per listed GPU,
      each with its own ``n`` pipelines (executor buffers, HIP stream, hipGraph) per frame size.
      Streams are assigned to replicas round-robin when they open (``session()``); replicas never
      communicate, so N GPUs serve N times the streams.
    * Frame sizes: the configured (H, W) keeps its pipelines; at most ``max_sizes`` other sizes have
      pipelines at once per replica (each holds full-size device buffers and captured graphs), the
      least recently used idle one is dropped for a new size, and a new size with every other size's
      pipelines busy is refused (the frame gets an error status) -- a client varying the frame size
      cannot grow device memory without bound.
    * ``session()`` gives a stream double-buffering: frame i+1 is staged and replayed on a second
      pipeline (own stream) while frame i's result is still on the device, so H2D, graph and D2H of
      consecutive frames overlap and the host tail of frame i overlaps the GPU work of frame i+1.
    """

    def __init__(self, model, K, depth_scale, H: int = 480, W: int = 640, size: int = 256, n: int = 2,
                 threshold: float = 0.5, graph: bool = True, geo_cfg: Optional[GeometryConfig] = None,
                 devices=None, rgb: bool = False, jpeg: bool = False, max_sizes: int = 3, batch: Optional[int] = None):
        self.model = model
        self.home_size = (H, W)
        self.max_sizes = max(0, max_sizes)
        self.rgb = rgb  # channel order of the frames this pool will be fed (graphs captured for it)
        self.args = dict(K=K, depth_scale=depth_scale, size=size, threshold=threshold, geo_cfg=geo_cfg)
        self.graph = graph
        self.n = max(1, n)
        self.gpu = _is_native(model)
        self.jpeg = jpeg and self.gpu  # GPU pipelines also fed JpegCoefs (their graph captured at build)
        home = _model_device(model)
        devs = [torch.device(d) for d in (devices or [home])]
        self.devices = devs
        self.replicas = [model if devs[i] == home and i == 0 else replicate_model(model, devs[i])
                         for i in range(len(devs))]
        self._pools: "collections.OrderedDict" = collections.OrderedDict()  # (r, H, W) -> Queue, LRU order
        self._mk_lock = threading.Lock()
        self._rr = 0
        self.sessions_opened = [0] * len(self.replicas)
        for r in range(len(self.replicas)):
            self._get(r, H, W)
        # cross-stream batching (BatchEngine): positions per batch (0: off; RDP_SERVE_BATCH). Frames of the
        # configured size from sessions of a replica that is serving >= 2 active streams go through it;
        # a lone stream keeps its double-buffered pipelines (no batching wait on its latency).
        if batch is None:
            batch = int(os.environ.get("RDP_SERVE_BATCH", "4"))
        self.batch_positions = batch if (self.gpu and graph and batch >= 2) else 0
        self.batchers = []
        if self.batch_positions:
            src = SRC_JPEG if self.jpeg else (SRC_RGB if rgb else SRC_BGR)
            self.batchers = [BatchEngine(self.replicas[r], H=H, W=W, device=self.devices[r], src=src,
                                         positions=self.batch_positions, **self.args) for r in range(len(self.replicas))]
        self._recent = [dict() for _ in self.replicas]  # replica -> {session id: last submit time}
        self.batch_active_s = 0.005
        for r, b in enumerate(self.batchers):
            b.target = (lambda r=r: self._active(r))

    def _active(self, r: int) -> int:
        """Sessions of replica ``r`` that submitted within the last ``batch_active_s``."""
        now = time.perf_counter()
        return sum(1 for t in list(self._recent[r].values()) if now - t <= self.batch_active_s)

    def _batcher(self, r: int, sid: int, shape) -> "Optional[BatchEngine]":
        """The replica's BatchEngine if this frame should be batched: configured frame size and at least two
        sessions of the replica submitted within the last ``batch_active_s``."""
        if not self.batchers or tuple(shape) != self.home_size:
            return None
        now = time.perf_counter()
        rec = self._recent[r]
        rec[sid] = now
        if len(rec) > 64:
            for k in [k for k, t in rec.items() if now - t > self.batch_active_s]:
                rec.pop(k, None)
        return self.batchers[r] if self._active(r) >= 2 else None

    def _new(self, r: int, H, W):
        m = self.replicas[r]
        if self.gpu:
            return FramePipeline(m, H=H, W=W, graph=self.graph, device=self.devices[r], rgb=self.rgb,
                                 jpeg=self.jpeg, **self.args)
        return CpuFramePipeline(m, H=H, W=W, **self.args)

    def _get(self, r: int, H, W) -> "queue.Queue":
        with self._mk_lock:
            key = (r, H, W)
            q = self._pools.get(key)
            if q is not None:
                self._pools.move_to_end(key)
                return q
            if (H, W) != self.home_size:
                other = [k for k in self._pools if k[0] == r and k[1:] != self.home_size]
                if len(other) >= self.max_sizes:
                    # drop the least recently used size whose pipelines are all idle (in the queue)
                    victim = next((k for k in other if self._pools[k].qsize() == self.n), None)
                    if victim is None:
                        raise RuntimeError(f"frame size {H}x{W}: {len(other)} other frame sizes are in flight "
                                           f"on this replica (max_sizes={self.max_sizes})")
                    del self._pools[victim]
            q = queue.Queue()
            for _ in range(self.n):
                q.put(self._new(r, H, W))
            self._pools[key] = q
            return q

    def session(self) -> "EngineSession":
        """A per-stream handle bound to the next replica (round-robin)."""
        with self._mk_lock:
            r = self._rr % len(self.replicas)
            self._rr += 1
            self.sessions_opened[r] += 1
        return EngineSession(self, r)

    @contextlib.contextmanager
    def exclusive(self):
        """Hold every pipeline of every replica (no frame in flight), e.g. while weights are swapped
        in place; yields the held pipelines and batch engines (all of them drained)."""
        with self._mk_lock:
            held = [(q, q.get()) for q in self._pools.values() for _ in range(self.n)]
            held_b = [b.hold() for b in self.batchers]
            try:
                yield [p for _, p in held] + list(self.batchers)
            finally:
                for b in self.batchers:
                    b.unhold()
                for q, p in held:
                    q.put(p)

    def load_state_dict(self, sd):
        """Hot reload: copy new weights into every replica, each with its own GPU current (call inside
        ``exclusive()``)."""
        for m, d in zip(self.replicas, self.devices):
            with _on(d):
                m.load_state_dict(sd)
                if hasattr(m, "refresh_weights"):
                    m.refresh_weights()

    @staticmethod
    def refresh_weights(pipelines):
        """After the shared weights changed (inside ``exclusive()``): refresh derived state."""
        for p in pipelines:
            p.refresh_weights()

    def process(self, color_bgr: np.ndarray, depth: np.ndarray) -> FrameResult:
        """One frame, synchronously, on the next replica."""
        s = self.session()
        s.submit(color_bgr, depth)
        return s.drain()[0][1]


class EngineSession:
    """One stream's view of the pool: up to ``depth`` frames in flight on its replica's pipelines.

    ``submit`` never blocks while this session holds a pipeline: if none is free it first collects
    its own oldest frame (returned to the caller), so concurrent sessions cannot deadlock."""

    def __init__(self, pool: EnginePool, replica: int, depth: int = 2):
        self.pool, self.replica, self.depth = pool, replica, max(1, depth)
        self.inflight: "collections.deque" = collections.deque()
        self.sid = id(self)

    def _batch_pos(self, b: "BatchEngine", out: list):
        """A position in ``b``'s open batch: without blocking if one is free, else after collecting this
        session's own frames (a session never waits on the pool while holding positions others wait on)."""
        pos = b._acquire(block=False)
        while pos is None and self.inflight:  # oldest first, only as many as needed
            out.append(self._collect_one())
            pos = b._acquire(block=False)
        return pos if pos is not None else b._acquire()

    def submit(self, color_bgr, depth, tag=None, rgb: bool = False) -> list:
        """Stage + enqueue a frame; returns [(tag, FrameResult | Exception)] of frames it had to collect.
        ``rgb``: the colour frame is in RGB order (else OpenCV BGR). ``depth`` may be a
        ``concurrent.futures.Future`` of the depth frame (the server's decode): the colour half of the
        frame is then enqueued first and the depth half when the future resolves."""
        out = []
        split = isinstance(depth, futures.Future)
        dshape = None if split else depth.shape[:2]
        if color_bgr.ndim != 3 or color_bgr.shape[2] != 3 or (dshape is not None and color_bgr.shape[:2] != dshape):
            if split:
                depth.cancel()
            out += self.drain()  # results stay in submission order
            out.append((tag, ValueError(f"colour {color_bgr.shape} and depth {dshape} frame sizes differ")))
            return out
        while len(self.inflight) >= self.depth:
            out.append(self._collect_one())
        b = None if split or isinstance(color_bgr, JpegCoefs) else self.pool._batcher(self.replica, self.sid,
                                                                                         color_bgr.shape[:2])
        if b is not None and b.src == (SRC_RGB if rgb else SRC_BGR):
            try:
                t = b.submit(color_bgr, depth, pos=self._batch_pos(b, out))
            except Exception as e:
                out += self.drain()
                out.append((tag, e))
                return out
            self.inflight.append((tag, b, t, "array"))
            return out
        try:
            q = self.pool._get(self.replica, *color_bgr.shape[:2])
        except RuntimeError as e:  # too many frame sizes in flight: this frame fails, the stream goes on
            if split:
                depth.cancel()
            out += self.drain()
            out.append((tag, e))
            return out
        try:
            p = q.get_nowait()
        except queue.Empty:
            while self.inflight:  # free our own pipelines before waiting on others'
                out.append(self._collect_one())
            p = q.get()
        try:
            if split:
                p.submit_color(color_bgr, rgb)
                try:
                    d = depth.result()
                    if d.shape[:2] != color_bgr.shape[:2]:
                        raise ValueError(f"colour {color_bgr.shape} and depth {d.shape} frame sizes differ")
                    p.submit_depth(d)
                except BaseException:
                    p.abort()
                    raise
            else:
                p.submit(color_bgr, depth, rgb)
        except BaseException as e:  # the pipeline goes back to its pool whatever was raised
            q.put(p)
            if not isinstance(e, Exception):
                raise
            out += self.drain()
            out.append((tag, e))
            return out
        self.inflight.append((tag, p, q))
        return out

    def submit_request(self, raw: bytes, tag=None):
        """``submit_encoded`` from a whole serialized AnalysisRequest (the server's raw-bytes handler)."""
        return self.submit_encoded(None, None, tag, raw=raw)

    def submit_encoded(self, color: bytes, depth: bytes, tag=None, raw: Optional[bytes] = None):
        """A request's encoded colour / depth bytes straight to a pipeline of the pool's configured size
        (FramePipeline.submit_encoded: decode + launch natively, no interpreter lock). Returns
        (collected, code): the frames it had to collect, and 0 when this frame is in flight -- else
        nothing of it is (1 / 2 / 3: decode it and ``submit`` instead)."""
        out = []
        while len(self.inflight) >= self.depth:
            out.append(self._collect_one())
        b = self.pool._batcher(self.replica, self.sid, self.pool.home_size)
        if b is not None and b.src == SRC_JPEG:
            try:
                pos = self._batch_pos(b, out)
                code, t = (b.submit_request(raw, pos=pos) if raw is not None
                           else b.submit_encoded(color, depth, pos=pos))
            except Exception as e:
                out += self.drain()
                out.append((tag, e))
                return out, 0
            if code == 0:
                self.inflight.append((tag, b, t, "encoded"))
            return out, code
        q = self.pool._get(self.replica, *self.pool.home_size)
        try:
            p = q.get_nowait()
        except queue.Empty:
            while self.inflight:
                out.append(self._collect_one())
            p = q.get()
        try:
            if not getattr(p, "encoded", False):
                code = 1
            else:
                code = p.submit_request(raw) if raw is not None else p.submit_encoded(color, depth)
        except BaseException as e:
            q.put(p)
            if not isinstance(e, Exception):
                raise
            out += self.drain()
            out.append((tag, e))
            return out, 0
        if code != 0:
            q.put(p)
            return out, code
        self.inflight.append((tag, p, q, True))
        return out, 0

    def submit_encoded_handle(self, color: bytes, depth: bytes, stop=None):
        """The server's reader-thread form of ``submit_encoded``: decode + launch one frame and return
        ``("t", handle)`` for ``collect_handle``, or ``("d", code)`` when nothing of it runs (as
        ``submit_encoded``'s codes). It never collects: it waits for a free pipeline / batch position
        instead, which the stream's handler thread frees as it collects the handles in order -- so frame
        i + 1 decodes while frame i is on the GPU or being collected. The caller bounds the handles it has
        outstanding (<= ``depth``). ``stop``: an Event that ends the wait for a pipeline (returns
        ``("d", 1)``)."""
        b = self.pool._batcher(self.replica, self.sid, self.pool.home_size)
        if b is not None and b.src == SRC_JPEG:
            code, t = b.submit_encoded(color, depth)  # blocks for a position while the batch frames are full
            return ("t", (b, t)) if code == 0 else ("d", code)
        q = self.pool._get(self.replica, *self.pool.home_size)
        while True:
            try:
                p = q.get(timeout=0.05)
                break
            except queue.Empty:
                if stop is not None and stop.is_set():
                    return ("d", 1)
        try:
            code = p.submit_encoded(color, depth) if getattr(p, "encoded", False) else 1
        except BaseException:
            q.put(p)
            raise
        if code != 0:
            q.put(p)
            return ("d", code)
        return ("t", (p, q))

    @staticmethod
    def collect_handle(handle):
        """The WireResult (or FrameResult / exception) of a ``submit_encoded_handle`` frame; its pipeline or
        batch position is free afterwards."""
        obj, x = handle
        try:
            if isinstance(obj, BatchEngine):
                return obj.collect_encoded(x)
            return obj.collect_encoded()
        except Exception as e:
            return e
        finally:
            if not isinstance(obj, BatchEngine):
                x.put(obj)

    def _collect_one(self):
        tag, p, q, *enc = self.inflight.popleft()
        if isinstance(p, BatchEngine):  # q: the frame's ticket, enc: its kind
            try:
                return tag, (p.collect_encoded(q) if enc[0] == "encoded" else p.collect(q))
            except Exception as e:
                return tag, e
        try:
            return tag, (p.collect_encoded() if enc else p.collect())
        except Exception as e:  # a failed frame must not take the pipeline with it
            return tag, e
        finally:
            q.put(p)

    def collect_oldest(self) -> list:
        return [self._collect_one()] if self.inflight else []

    def drain(self) -> list:
        out = []
        while self.inflight:
            out.append(self._collect_one())
        return out

    def close(self) -> None:
        """Give every pipeline this session holds back to its pool without building results (a stream
        that ended early: client cancel, transport error, abort). Idempotent."""
        while self.inflight:
            _, p, q, *_enc = self.inflight.popleft()
            if isinstance(p, BatchEngine):
                try:
                    p.collect(q)  # waits for its batch, releases the position
                except Exception:
                    pass
                continue
            try:
                p.wait_idle()
            except Exception:  # the pipeline goes back either way
                pass
            finally:
                q.put(p)


def _model_device(model) -> torch.device:
    if _is_native(model):
        return model.store.device
    try:
        return next(model.parameters()).device
    except (StopIteration, AttributeError):
        return torch.device("cpu")


def _is_native(model) -> bool:
    try:
        from ..models.unet import UNetNative
        return isinstance(model, UNetNative)
    except Exception:
        return False


def smoke_frame(model, device) -> FrameResult:
    """One synthetic 480x640 frame through the native pipeline (used by __graft_entry__.smoke)."""
    from ..data.synthetic import DEFAULT_K, make_scene
    sc = make_scene(0)
    p = FramePipeline(model, DEFAULT_K, 0.001, graph=True, device=device)
    r = p.process(sc.color, sc.depth)
    assert r.mask.shape == (480, 640) and 0.0 <= r.coverage <= 100.0
    return r

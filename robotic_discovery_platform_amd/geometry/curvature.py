"""Curvature profile of the segmented actuator: the native pipeline.

API-compatible with ``/root/reference/pkg/geometry_utils.py`` (``compute_curvature_profile(mask,
depth_image, intrinsics, depth_scale) -> CurvatureResult`` with ``Point`` / ``CurvatureResult``
dataclasses, same early-exit and failure semantics), executed MI355X-first:

  GPU (csrc/geometry.hip, graph-capturable):  masked-depth deprojection + row-major stream
      compaction (fp64) -> x min/max -> 50-bin top-5 %-by-y edge selection (radix select, exact
      tie-breaking) -> packed edge points
  GPU (csrc/geo_spline.hip, graph-capturable):  per-bin sort by x, FITPACK-equivalent parametric
      smoothing spline (s = 0.1, k = 3; banded normal equations reduced over the points in
      parallel, FITPACK's knot / smoothing-parameter control flow on one thread), 100-sample
      splev + curvature |r' x r''| / |r'|^3 -> a 308-double result (status, kappa mean/max, points)
  host (csrc/spline.cpp):  the exact FITPACK port -- the CPU path, the test oracle, and the
      fallback for the rare fit that needs more than the device's 64 coefficients per dimension
"""
from __future__ import annotations

from dataclasses import dataclass, field
import itertools
from typing import List, Optional, Tuple

import numpy as np
import torch

from ..config import GeometryConfig


@dataclass(slots=True)  # one per spline sample, built on every served frame
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
    n_points: int = 0
    n_edge_points: int = 0


def sort_edges(edges: np.ndarray) -> np.ndarray:
    """edges [E, 4] (x, y, z, index) -> points sorted by x asc, then y desc, then index asc
    (= a stable sort by x of the per-bin, y-descending concatenation the reference builds)."""
    order = np.lexsort((edges[:, 3], -edges[:, 1], edges[:, 0]))
    return np.ascontiguousarray(edges[order, :3])


def fit_edges(pts_sorted: np.ndarray, cfg: GeometryConfig, n_points: int) -> CurvatureResult:
    from ..ops import native
    C = native()
    E = pts_sorted.shape[0]
    if E < cfg.min_edge_points:
        return CurvatureResult(status="too_few_edge_points", n_points=n_points, n_edge_points=E)
    ier, mk, xk, spts, fp, n = C.fit_curvature(torch.from_numpy(pts_sorted), cfg.smoothing, cfg.spline_degree,
                                               cfg.num_samples, cfg.deriv_eps)
    if ier == 10:  # FITPACK "invalid input" == scipy ValueError -> empty result (reference :95-97)
        return CurvatureResult(status="fit_failed", n_points=n_points, n_edge_points=E)
    p = spts.numpy()
    return CurvatureResult(float(mk), float(xk), [Point(float(a), float(b), float(c)) for a, b, c in p], "ok",
                           n_points, E)


# device result status codes (csrc/geo_spline.hip)
_DEV_STATUS = {0: "ok", 1: "too_few_points", 2: "too_few_edge_points", 3: "fit_failed"}
DEV_NEEDS_HOST = 4


def coverage_from_device(res: np.ndarray, cfg: GeometryConfig) -> int:
    """Mask pixel count carried in the device result (serving form; -1 if not produced)."""
    return int(res[8 + 3 * cfg.num_samples])


def result_from_device(res: np.ndarray, cfg: GeometryConfig) -> Optional[CurvatureResult]:
    """CurvatureResult from the device result vector; None when the fit must finish on the host."""
    st = int(res[0])
    if st == DEV_NEEDS_HOST:
        return None
    E, npts = int(res[6]), int(res[7])
    if st != 0:
        return CurvatureResult(status=_DEV_STATUS.get(st, "fit_failed"), n_points=npts,
                               n_edge_points=E if st != 1 else 0)
    p = res[8:8 + 3 * cfg.num_samples].reshape(-1, 3).tolist()  # Python floats in one C pass
    return CurvatureResult(float(res[4]), float(res[5]), list(itertools.starmap(Point, p)), "ok", npts, E)


def edges_numpy(mask, depth, K, scale, cfg: GeometryConfig) -> Tuple[np.ndarray, int]:
    """CPU edge extraction with the kernels' exact semantics (used where no GPU is present)."""
    v, u = np.nonzero(mask > 0)
    z = depth[v, u].astype(np.float64) * scale
    keep = z > 0
    v, u, z = v[keep], u[keep], z[keep]
    n = len(z)
    if n < cfg.min_points:
        return np.zeros((0, 4)), n
    x = (u - K[0, 2]) * z / K[0, 0]
    y = (v - K[1, 2]) * z / K[1, 1]
    idx = np.arange(n, dtype=np.float64)
    lo, hi = x.min(), x.max()
    w = (hi - lo) / cfg.num_bins
    if not w > 0:
        return np.zeros((0, 4)), n
    b = np.clip(np.floor((x - lo) / w), 0, cfg.num_bins - 1).astype(np.int64)
    out = []
    for i in range(cfg.num_bins):
        sel = np.nonzero(b == i)[0]
        if len(sel):
            k = max(1, int(len(sel) * cfg.top_k_percent))
            o = sel[np.lexsort((sel, -y[sel]))][:k]
            out.append(np.stack([x[o], y[o], z[o], idx[o]], 1))
    return (np.concatenate(out) if out else np.zeros((0, 4))), n


class GeometryEngine:
    """Device buffers + launch for one camera resolution (one per serving engine / stream)."""

    def __init__(self, H: int, W: int, device: torch.device, cfg: Optional[GeometryConfig] = None,
                 ecap: Optional[int] = None):
        from ..ops import native
        self.C = native()
        self.cfg = cfg or GeometryConfig()
        self.H, self.W, self.dev = H, W, device
        nblk = self.C.geo_nblocks(H)
        self.work_i = torch.zeros(self.C.geo_work_ints(H, W), dtype=torch.int32, device=device)
        self.work_d = torch.zeros(2 * nblk, dtype=torch.float64, device=device)
        self.pts = torch.zeros(H * W * 4, dtype=torch.float64, device=device)
        self.npts = torch.zeros(1, dtype=torch.int32, device=device)
        kcap = max(1, int(H * W * self.cfg.top_k_percent) + 1)
        self.out = torch.zeros(self.cfg.num_bins, kcap, 4, dtype=torch.float64, device=device)
        self.kout = torch.zeros(self.cfg.num_bins, dtype=torch.int32, device=device)
        # upper bound of sum_b max(1, int(n_b * top)) over <= H*W points: never truncates
        ecap = ecap or (self.cfg.num_bins + int(H * W * self.cfg.top_k_percent) + 1)
        self.edges = torch.zeros(ecap, 4, dtype=torch.float64, device=device)
        self.hdr = torch.zeros(1, dtype=torch.int32, device=device)
        # on-device spline stage: x-sorted edge points, merge scratch, chord parameters, result
        self.sorted = torch.zeros(ecap, 3, dtype=torch.float64, device=device)
        self.gperm = torch.zeros(2 * ecap, dtype=torch.int32, device=device)
        self.u = torch.zeros(ecap, dtype=torch.float64, device=device)
        self.res = torch.zeros(self.C.geo_spline_res_len(self.cfg.num_samples), dtype=torch.float64, device=device)
        self.cov = torch.zeros(nblk, dtype=torch.int32, device=device)

    def launch(self, mask_dev: torch.Tensor, depth_dev: torch.Tensor, K: np.ndarray, scale: float):
        """Enqueue the edge extraction on the current stream (no host sync; graph-capturable)."""
        c = self.cfg
        self.C.geo_edges(mask_dev, depth_dev, float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2]),
                         float(scale), self.work_i, self.work_d, self.pts, self.npts, self.out, self.kout, c.num_bins,
                         c.top_k_percent, c.min_points, self.edges, self.hdr)
        self._serving_form = False

    def launch_frame(self, m256_dev: torch.Tensor, mask_out: torch.Tensor, depth_dev: torch.Tensor, K: np.ndarray,
                     scale: float, mask_host: Optional[torch.Tensor] = None, host_copy_in_spline: bool = False):
        """Serving form: ``mask_out`` (H x W) is produced here by nearest-upsampling the model-resolution
        mask ``m256_dev`` (no separate upsample kernel), with the coverage count per row block, and no
        packed edge list; follow with ``launch_spline()`` (its result then carries the coverage).
        ``mask_host``: a host-memory copy of the mask (no read-back copy), written by the mask kernel, or
        with ``host_copy_in_spline`` by blocks of the next ``launch_spline()`` beside its single fit block
        (off the critical path: in the mask kernel the PCIe writes lengthened it by ~4.5 us)."""
        c = self.cfg
        defer = host_copy_in_spline and mask_host is not None and mask_out.numel() % 4 == 0
        self.C.geo_edges(mask_out, depth_dev, float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2]),
                         float(scale), self.work_i, self.work_d, self.pts, self.npts, self.out, self.kout, c.num_bins,
                         c.top_k_percent, c.min_points, None, None, m256_dev, self.cov, self.sorted, self.gperm,
                         None if defer else mask_host)
        self._host_copy = (mask_out, mask_host) if defer else None
        self._serving_form = True  # the select kernel also wrote the x-sorted edge points

    def launch_spline(self, res_out: Optional[torch.Tensor] = None):
        """Enqueue the on-device spline stage after ``launch`` (no host sync; graph-capturable).
        ``res_out``: where the result vector goes instead of ``self.res`` (e.g. host memory the kernel
        writes directly: nothing on the device reads it back)."""
        c = self.cfg
        serving = getattr(self, "_serving_form", False)
        self.C.geo_spline(self.out, self.kout, self.npts, self.sorted, self.gperm, self.u,
                          self.res if res_out is None else res_out, c.smoothing,
                          c.spline_degree, c.num_samples, c.deriv_eps, c.min_points, c.min_edge_points,
                          self.cov if serving else None, presorted=serving,
                          **({"mask": hc[0], "mask_host": hc[1]} if (hc := getattr(self, "_host_copy", None)) else {}))
        self._host_copy = None

    def finish_device(self, res_host: np.ndarray) -> CurvatureResult:
        """Result of ``launch_spline`` (``res`` read back); a fit beyond the device capacity is redone
        on the host from the device-sorted edge points (synchronous read-back, rare)."""
        r = result_from_device(res_host, self.cfg)
        if r is not None:
            return r
        E, npts = int(res_host[6]), int(res_host[7])
        return fit_edges(self.sorted[:E].cpu().numpy(), self.cfg, npts)

    def finish(self, edges_host: np.ndarray, E: int, n_points: int) -> CurvatureResult:
        if n_points < self.cfg.min_points:
            return CurvatureResult(status="too_few_points", n_points=n_points)
        return fit_edges(sort_edges(edges_host[:E]), self.cfg, n_points)


def compute_curvature_profile(mask: np.ndarray, depth_image: np.ndarray, intrinsics: np.ndarray,
                              depth_scale: float, cfg: Optional[GeometryConfig] = None,
                              device: Optional[torch.device] = None, spline: str = "device") -> CurvatureResult:
    """Reference-signature entry point (numpy in, CurvatureResult out). On a GPU the spline stage
    runs on the device (``spline="device"``) or on the host from the device's edge points
    (``spline="host"``, the FITPACK-exact oracle path)."""
    cfg = cfg or GeometryConfig()
    K = np.asarray(intrinsics, dtype=np.float64)
    use_gpu = torch.cuda.is_available() if device is None else torch.device(device).type == "cuda"
    if not use_gpu:
        edges, n = edges_numpy(mask, depth_image, K, depth_scale, cfg)
        if n < cfg.min_points:
            return CurvatureResult(status="too_few_points", n_points=n)
        return fit_edges(sort_edges(edges), cfg, n)
    dev = torch.device(device) if device is not None else torch.device("cuda")
    H, W = mask.shape
    eng = _engine_cache(H, W, dev, cfg)
    m = torch.from_numpy(np.ascontiguousarray(mask.astype(np.uint8))).to(dev)
    d = torch.from_numpy(np.ascontiguousarray(depth_image.astype(np.uint16)).view(np.int16)).to(dev)
    eng.launch(m, d, K, depth_scale)
    if spline == "device":
        eng.launch_spline()
        return eng.finish_device(eng.res.cpu().numpy())
    n = int(eng.npts.item())
    E = int(eng.hdr.item())
    return eng.finish(eng.edges[:min(E, eng.edges.shape[0])].cpu().numpy(), E, n)


_ENGINES = {}


def _engine_cache(H, W, dev, cfg):
    key = (H, W, str(dev), cfg.num_bins, cfg.top_k_percent, cfg.min_points)
    if key not in _ENGINES:
        _ENGINES[key] = GeometryEngine(H, W, dev, cfg)
    return _ENGINES[key]

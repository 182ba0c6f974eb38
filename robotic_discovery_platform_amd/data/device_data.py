"""Device-resident training data (MI355X: 288 GB HBM per GPU).

The reference's ``SegmentationDataset`` (``/root/reference/scripts/train_segmenter.py:66-100``)
decodes, converts BGR->RGB and INTER_AREA-resizes every colour image and INTER_NEAREST-resizes
every mask on the host, per sample, per epoch, on the training thread (``num_workers=0``). Here the
processed dataset is built ONCE on the GPU and kept there as u8 NHWC tensors (192 KiB per 256x256
RGB sample + 64 KiB per mask), so an epoch is pure device work: index_select of the shuffled batch,
u8 -> float /255 in the executor's input copy, and the training step.

Build: host threads decode the files (PIL releases the GIL); each full-size u8 image is uploaded and
resized by ``resize_area_u8`` (csrc/data_kernels.hip, fp64 INTER_AREA + BGR->RGB) and each mask by
the nearest-neighbour kernel, straight into its slot of the resident tensors.
"""
from __future__ import annotations

from concurrent import futures
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from .image_io import _area_weights, resize_area, resize_nearest, bgr2rgb


def area_tables(n_in: int, n_out: int, maxtap: int):
    """(start[n_out] i32, size[n_out] i32, weights[n_out * maxtap] f64) of the INTER_AREA weights."""
    w = _area_weights(n_in, n_out)
    start = np.zeros(n_out, np.int32)
    size = np.zeros(n_out, np.int32)
    tab = np.zeros((n_out, maxtap), np.float64)
    for o in range(n_out):
        nz = np.nonzero(w[o])[0]
        lo, hi = int(nz[0]), int(nz[-1]) + 1
        if hi - lo > maxtap:
            raise ValueError(f"INTER_AREA {n_in}->{n_out} needs {hi - lo} taps > {maxtap}")
        start[o], size[o] = lo, hi - lo
        tab[o, : hi - lo] = w[o, lo:hi]
    return start, size, tab.reshape(-1)


class _Tables:
    def __init__(self, device):
        self.device = device
        self.cache = {}

    def get(self, n_in, n_out):
        key = (n_in, n_out)
        if key not in self.cache:
            from ..ops import native
            s, n, w = area_tables(n_in, n_out, native().area_maxtap())
            self.cache[key] = tuple(torch.from_numpy(a).to(self.device) for a in (s, n, w))
        return self.cache[key]


def resize_area_gpu(img: torch.Tensor, size: Tuple[int, int], swap_rb: bool = False, out: Optional[torch.Tensor] = None,
                    tables: Optional[_Tables] = None) -> torch.Tensor:
    """cv2.resize(INTER_AREA) (downscale) of a u8 HxWxC device tensor; ``swap_rb``: BGR -> RGB too."""
    from ..ops import native
    W, H = size
    h, w, c = img.shape
    if W > w or H > h:
        raise ValueError("resize_area_gpu downsamples only (the reference's 640x480 -> 256x256)")
    tables = tables or _Tables(img.device)
    ys, yn, yw = tables.get(h, H)
    xs, xn, xw = tables.get(w, W)
    out = out if out is not None else torch.empty(H, W, c, dtype=torch.uint8, device=img.device)
    native().resize_area_u8(img, ys, yn, yw, xs, xn, xw, int(swap_rb), out)
    return out


def resize_nearest_gpu(m: torch.Tensor, size: Tuple[int, int], out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """cv2 INTER_NEAREST of a u8 HxW device tensor (csrc/serve_kernels.hip mask_upsample)."""
    from ..ops import native
    W, H = size
    out = out if out is not None else torch.empty(H, W, dtype=torch.uint8, device=m.device)
    cnt = torch.zeros(1, dtype=torch.int32, device=m.device)
    native().mask_upsample(m.contiguous(), out, cnt)
    return out


def build_device_dataset(ds, indices: Sequence[int], device: torch.device, size: Tuple[int, int] = (256, 256),
                         workers: int = 8) -> Tuple[torch.Tensor, torch.Tensor]:
    """Resident (x [N,H,W,3] u8 RGB, y [N,H,W] u8) on ``device`` for ``ds[indices]``.

    ``ds`` provides ``raw_arrays(i) -> (colour BGR u8 HxWx3 at file size, mask u8 HxW)``; on a CPU
    device the host resizes (the numpy oracle) are used instead of the kernels."""
    W, H = size
    n = len(indices)
    x = torch.empty(n, H, W, 3, dtype=torch.uint8, device=device)
    y = torch.empty(n, H, W, dtype=torch.uint8, device=device)
    if n == 0:
        return x, y
    gpu = device.type == "cuda"
    tables = _Tables(device) if gpu else None
    with futures.ThreadPoolExecutor(max_workers=workers) as ex:
        for j, (img, mask) in enumerate(ex.map(ds.raw_arrays, list(indices))):
            if gpu and (img.shape[0] < H or img.shape[1] < W):  # upscaling: the host path (bilinear)
                x[j].copy_(torch.from_numpy(resize_area(bgr2rgb(img), size)))
                y[j].copy_(torch.from_numpy(resize_nearest(mask, size)))
            elif gpu:
                if img.shape[0] == H and img.shape[1] == W:
                    x[j].copy_(torch.from_numpy(np.ascontiguousarray(img[..., ::-1])))
                else:
                    resize_area_gpu(torch.from_numpy(img).to(device, non_blocking=False), size, swap_rb=True,
                                    out=x[j], tables=tables)
                resize_nearest_gpu(torch.from_numpy(np.ascontiguousarray(mask)).to(device), size, out=y[j])
            else:
                x[j].copy_(torch.from_numpy(resize_area(bgr2rgb(img), size)))
                y[j].copy_(torch.from_numpy(resize_nearest(mask, size)))
    return x, y


_LUT = {}


def _u8_lut(device) -> torch.Tensor:
    """v / 255 for v in 0..255, divided in fp64 and rounded to fp32 -- exactly the reference's
    ``image / 255.0`` (numpy float64) followed by ``.float()`` (a GPU tensor division by a scalar
    multiplies by the reciprocal and can be 1 ulp off)."""
    key = str(device)
    if key not in _LUT:
        _LUT[key] = (torch.arange(256, dtype=torch.float64) / 255.0).to(torch.float32).to(device)
    return _LUT[key]


def batch_to_float(xb: torch.Tensor, yb: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """u8 NHWC RGB + u8 NHW mask -> (float NCHW /255, float N1HW /255): the reference's item format."""
    lut = _u8_lut(xb.device)
    x = lut.index_select(0, xb.reshape(-1).int()).view(xb.shape).permute(0, 3, 1, 2)
    y = lut.index_select(0, yb.reshape(-1).int()).view(yb.shape).unsqueeze(1)
    return x, y

"""Baseline-JPEG decode split between the host (entropy decode) and the GPU (pixels).

The reference server decodes every colour frame with ``cv2.imdecode(IMREAD_COLOR)``
(``/root/reference/services/vision_analysis/server.py:117``): libjpeg's Huffman decode, ISLOW
integer IDCT, "fancy" chroma upsampling and fixed-point YCbCr -> RGB, all on one CPU thread. Here:

* ``decode_coefs`` (``csrc/jpeg.cpp``): Huffman-decodes the scan into quantised DCT coefficient planes
  without the GIL; the restart segments of a JPEG written with restart markers (our client writes one
  per MCU row, ``serve/client.py``: still a standard baseline JPEG) decode in parallel on a small
  native thread pool.
* ``csrc/serve_kernels.hip`` (``jpeg_to_rgb``, inside the per-frame graph): dequantisation + IDCT +
  upsampling + colour conversion on the GPU, straight into the frame buffer the preprocess reads.

``coefs_to_rgb_reference`` is the same pixel math in NumPy (the CPU oracle of the GPU kernels; tests
check it against PIL's libjpeg decode). Unsupported streams (progressive, arithmetic, 12-bit ...) make
``decode_coefs`` return None and the caller decodes with PIL.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np


@dataclass
class JpegCoefs:
    """One entropy-decoded frame: ``meta`` int32[32 + 192] (geometry, then the three quantisation
    tables in natural order; bindings.cpp jpeg_decode has the layout) and the int16 coefficient
    planes. A stand-in for the HxWx3 array it decodes to (``shape`` / ``ndim``)."""
    meta: "object"   # torch int32 [224]
    coefs: "object"  # torch int16 [n]
    ndim = 3

    @property
    def geo(self):
        return self.meta[:32]

    @property
    def qt(self):
        return self.meta[32:]

    @property
    def width(self) -> int:
        return int(self.meta[0])

    @property
    def height(self) -> int:
        return int(self.meta[1])

    @property
    def blocks(self) -> int:
        return int(self.meta[5])

    @property
    def shape(self):  # (H, W, 3), like the decoded array it stands for
        return (self.height, self.width, 3)


def decode_coefs(data: bytes, parallel: bool = True, pin: bool = False) -> Optional[JpegCoefs]:
    """Entropy-decode a baseline JPEG (None: not a stream the native decoder takes -> use PIL).
    ``pin``: outputs in pinned host memory (the GPU pipeline copies them asynchronously)."""
    try:
        from ..ops import native
        C = native(build_if_missing=False)
    except Exception:  # pragma: no cover
        return None
    if C is None or not hasattr(C, "jpeg_decode"):
        return None
    r = C.jpeg_decode(bytes(data), parallel, pin)
    if r is None:
        return None
    return JpegCoefs(*r)


# ---------------------------------------------------------------------------------------- oracle
_F = dict(f0_298631336=2446, f0_390180644=3196, f0_541196100=4433, f0_765366865=6270, f0_899976223=7373,
          f1_175875602=9633, f1_501321110=12299, f1_847759065=15137, f1_961570560=16069, f2_053119869=16819,
          f2_562915447=20995, f3_072711026=25172)


def _idct_1d(v):
    """ISLOW 1-D pass over axis -1 of an int64 array [..., 8]; returns (even[4], odd[4]) pre-descale."""
    f = _F
    z2, z3 = v[..., 2], v[..., 6]
    z1 = (z2 + z3) * f["f0_541196100"]
    t2 = z1 + z3 * -f["f1_847759065"]
    t3 = z1 + z2 * f["f0_765366865"]
    t0 = (v[..., 0] + v[..., 4]) << 13
    t1 = (v[..., 0] - v[..., 4]) << 13
    e = [t0 + t3, t1 + t2, t1 - t2, t0 - t3]
    a0, a1, a2, a3 = v[..., 7], v[..., 5], v[..., 3], v[..., 1]
    z1, z2, z3, z4 = a0 + a3, a1 + a2, a0 + a2, a1 + a3
    z5 = (z3 + z4) * f["f1_175875602"]
    a0, a1, a2, a3 = a0 * f["f0_298631336"], a1 * f["f2_053119869"], a2 * f["f3_072711026"], a3 * f["f1_501321110"]
    z1, z2 = z1 * -f["f0_899976223"], z2 * -f["f2_562915447"]
    z3, z4 = z3 * -f["f1_961570560"] + z5, z4 * -f["f0_390180644"] + z5
    o = [a0 + z1 + z3, a1 + z2 + z4, a2 + z2 + z3, a3 + z1 + z4]
    return e, o


def _combine(e, o, shift):
    r = 1 << (shift - 1)
    rows = [e[0] + o[3], e[1] + o[2], e[2] + o[1], e[3] + o[0], e[3] - o[0], e[2] - o[1], e[1] - o[2], e[0] - o[3]]
    return np.stack([(x + r) >> shift for x in rows], axis=-1)


def idct_blocks(blocks: np.ndarray, q: np.ndarray) -> np.ndarray:
    """[n, 64] quantised int16 blocks (natural order) + [64] table -> [n, 8, 8] u8 samples (ISLOW)."""
    x = blocks.astype(np.int64).reshape(-1, 8, 8) * q.astype(np.int64).reshape(8, 8)
    e, o = _idct_1d(np.swapaxes(x, 1, 2))          # columns: [n, col, row]
    ws = _combine(e, o, 13 - 2)                     # [n, col, out row]
    e, o = _idct_1d(np.swapaxes(ws, 1, 2))          # rows: [n, row, col]
    out = _combine(e, o, 13 + 2 + 3) + 128
    return np.clip(out, 0, 255).astype(np.uint8)


def _fancy(plane: np.ndarray, hr: int, vr: int, dsh: int, dsw: int, H: int, W: int) -> np.ndarray:
    p = plane[:dsh, :dsw].astype(np.int64)
    if hr == 1 and vr == 1:
        return p[:H, :W]
    if hr == 2 and vr == 1:
        left = np.concatenate([p[:, :1], p[:, :-1]], 1)
        right = np.concatenate([p[:, 1:], p[:, -1:]], 1)
        out = np.empty((p.shape[0], 2 * p.shape[1]), np.int64)
        out[:, 0::2] = (3 * p + left + 1) >> 2
        out[:, 1::2] = (3 * p + right + 2) >> 2
        return out[:H, :W]
    if hr == 2 and vr == 2:
        up = np.concatenate([p[:1], p[:-1]], 0)
        dn = np.concatenate([p[1:], p[-1:]], 0)
        out = np.empty((2 * p.shape[0], 2 * p.shape[1]), np.int64)
        for v, nb in ((0, up), (1, dn)):
            cs = 3 * p + nb
            left = np.concatenate([cs[:, :1], cs[:, :-1]], 1)
            right = np.concatenate([cs[:, 1:], cs[:, -1:]], 1)
            out[v::2, 0::2] = (3 * cs + left + 8) >> 4
            out[v::2, 1::2] = (3 * cs + right + 7) >> 4
        return out[:H, :W]
    raise NotImplementedError(f"chroma ratio {hr}x{vr}")


def coefs_to_rgb_reference(jc: JpegCoefs) -> np.ndarray:
    """NumPy oracle of the GPU pixel stage: HxWx3 uint8 RGB."""
    g = jc.geo.numpy().astype(np.int64)
    co = jc.coefs.numpy()
    qt = jc.qt.numpy().reshape(3, 64)
    W, H, nc, hmax, vmax = (int(v) for v in g[:5])
    planes = []
    for c in range(nc):
        h, v, bw, bh, b0 = (int(x) for x in g[8 + 8 * c: 13 + 8 * c])
        blk = co[b0 * 64:(b0 + bw * bh) * 64].reshape(bw * bh, 64)
        px = idct_blocks(blk, qt[c]).reshape(bh, bw, 8, 8).transpose(0, 2, 1, 3).reshape(bh * 8, bw * 8)
        planes.append((px, h, v, int(g[14 + 8 * c]), int(g[15 + 8 * c])))
    y = planes[0][0][:H, :W].astype(np.int64)
    if nc == 1:
        return np.repeat(y[..., None], 3, axis=2).astype(np.uint8)
    cb = _fancy(planes[1][0], hmax // planes[1][1], vmax // planes[1][2], planes[1][4], planes[1][3], H, W) - 128
    cr = _fancy(planes[2][0], hmax // planes[2][1], vmax // planes[2][2], planes[2][4], planes[2][3], H, W) - 128
    r = y + ((91881 * cr + 32768) >> 16)
    gg = y + ((-22554 * cb + 32768 - 46802 * cr) >> 16)
    b = y + ((116130 * cb + 32768) >> 16)
    return np.clip(np.stack([r, gg, b], -1), 0, 255).astype(np.uint8)

"""Image codecs and OpenCV-semantics resizes without OpenCV (cv2 is not available).

Reference uses of OpenCV:
  * ``cv2.imencode('.jpg', bgr)`` / ``cv2.imencode('.png', depth_u16)`` (client.py:65-67),
    ``cv2.imdecode(..., IMREAD_COLOR / IMREAD_UNCHANGED)`` (server.py:117-118),
    ``cv2.imencode('.png', mask*255)`` (server.py:142).
  * ``cv2.resize(INTER_AREA)`` for training images, ``INTER_NEAREST`` for masks
    (train_segmenter.py:86,90) and for the served mask (server.py:125).
Codecs: grayscale 8/16-bit PNG (depth in, mask out: the per-frame serving codecs) go through the
native zlib codec (csrc/codecs.cpp, no GIL held); JPEG and every other PNG flavour through PIL.
Arrays keep OpenCV's conventions: colour images are HxWx3 uint8 **BGR**, depth is HxW uint16.
"""
from __future__ import annotations

import io
from typing import Tuple

import numpy as np
from PIL import Image, ImageOps


# ----------------------------------------------------------------------------- codecs
def encode_jpeg(bgr: np.ndarray, quality: int = 95, restart_rows: int = 0) -> bytes:
    """Baseline JPEG of a BGR frame (cv2.imencode('.jpg') equivalent). ``restart_rows`` > 0 puts a
    restart marker after every that many MCU rows -- still a standard baseline stream that any decoder
    reads; the server's native decoder (data/jpeg.py) decodes the segments in parallel."""
    rgb = np.ascontiguousarray(bgr[..., ::-1])
    buf = io.BytesIO()
    kw = {"restart_marker_rows": int(restart_rows)} if restart_rows > 0 else {}
    Image.fromarray(rgb, "RGB").save(buf, format="JPEG", quality=quality, **kw)
    return buf.getvalue()


_PNG_SIG = b"\x89PNG\r\n\x1a\n"


def _native():
    try:
        from ..ops import native
        return native()
    except Exception:  # pragma: no cover - no extension: PIL only
        return None


def encode_png(arr: np.ndarray, compress_level: int = 6, bands: int = 1) -> bytes:
    """PNG of uint8 gray, uint8 BGR (stored as RGB) or uint16 gray (lossless 16-bit). Grayscale goes
    through the native encoder; ``bands`` > 1 writes a banded stream (an ordinary PNG for every reader,
    which the native decoder inflates band-parallel: csrc/codecs.cpp)."""
    if arr.ndim == 2 and arr.dtype in (np.uint8, np.uint16) and 0 <= compress_level <= 9:
        C = _native()
        if C is not None:
            import torch
            a = np.ascontiguousarray(arr)
            return C.png_encode(torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else a),
                                int(compress_level), max(1, int(bands)))
    buf = io.BytesIO()
    kw = dict(format="PNG", compress_level=compress_level)
    if arr.dtype == np.uint16:
        Image.fromarray(np.ascontiguousarray(arr)).save(buf, **kw)  # uint16 -> mode I;16
    elif arr.ndim == 3:
        Image.fromarray(np.ascontiguousarray(arr[..., ::-1]), "RGB").save(buf, **kw)
    else:
        Image.fromarray(np.ascontiguousarray(arr.astype(np.uint8)), "L").save(buf, **kw)
    return buf.getvalue()


def decode_image(data: bytes, color: bool = True, order: str = "BGR") -> np.ndarray:
    """IMREAD_COLOR -> HxWx3 uint8 BGR (``order="RGB"``: RGB, skipping the channel flip for consumers
    that take either order); color=False -> IMREAD_UNCHANGED (uint8 or uint16 gray)."""
    if not color and data[:8] == _PNG_SIG:
        C = _native()
        t = C.png_decode(bytes(data)) if C is not None else None
        if t is not None:
            a = t.numpy()
            return a.view(np.uint16) if a.dtype == np.int16 else a
    im = Image.open(io.BytesIO(data))
    if color:
        im.load()
        if im.getexif().get(0x0112, 1) != 1:  # cv2.imdecode(IMREAD_COLOR) applies the EXIF orientation
            im = ImageOps.exif_transpose(im)
        rgb = np.asarray(im if im.mode == "RGB" else im.convert("RGB"))
        return rgb if order == "RGB" else rgb[..., ::-1].copy()
    if im.mode in ("I;16", "I;16B", "I;16L", "I"):
        return np.asarray(im, dtype=np.uint16).copy() if im.mode != "I" else np.asarray(im).astype(np.uint16)
    if im.mode == "L":
        return np.asarray(im).copy()
    return np.asarray(im.convert("RGB"))[..., ::-1].copy()


def imread(path: str, color: bool = True) -> np.ndarray:
    if str(path).endswith(".npy"):
        return np.load(path, allow_pickle=False)
    with open(path, "rb") as f:
        return decode_image(f.read(), color)


def imread_gray(path: str) -> np.ndarray:
    im = Image.open(path)
    if im.mode not in ("L",):
        im = im.convert("L")
    return np.asarray(im).copy()


def imwrite(path: str, arr: np.ndarray) -> None:
    p = str(path)
    if p.endswith(".npy"):
        np.save(p, arr)
    elif p.lower().endswith((".jpg", ".jpeg")):
        open(p, "wb").write(encode_jpeg(arr))
    else:
        open(p, "wb").write(encode_png(arr))


def bgr2rgb(img: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(img[..., ::-1])


# ----------------------------------------------------------------------------- resizes
def _area_weights(n_in: int, n_out: int) -> np.ndarray:
    """OpenCV INTER_AREA weight matrix (n_out x n_in): overlap of [o*s, (o+1)*s) with input pixels / s."""
    s = n_in / n_out
    a = np.arange(n_out)[:, None] * s
    b = a + s
    i = np.arange(n_in)[None, :]
    ov = np.clip(np.minimum(b, i + 1) - np.maximum(a, i), 0.0, None)
    ov[ov < 1e-12] = 0.0
    return ov / s


def resize_area(img: np.ndarray, size: Tuple[int, int]) -> np.ndarray:
    """cv2.resize(img, (W, H), interpolation=INTER_AREA) for downscaling (uint8 result, cvRound)."""
    W, H = size
    h, w = img.shape[:2]
    if W > w or H > h:
        return resize_bilinear(img, size)
    wy, wx = _area_weights(h, H), _area_weights(w, W)
    x = img.astype(np.float64)
    if x.ndim == 2:
        out = wy @ x @ wx.T
    else:  # separable: rows then columns (two BLAS matmuls)
        t = np.tensordot(wy, x, axes=(1, 0))           # (H, w, c)
        out = np.tensordot(t, wx, axes=(1, 1)).transpose(0, 2, 1)  # (H, W, c)
    if img.dtype == np.uint8:
        return np.clip(np.rint(out), 0, 255).astype(np.uint8)
    return out.astype(img.dtype)


def resize_nearest(img: np.ndarray, size: Tuple[int, int]) -> np.ndarray:
    """cv2 INTER_NEAREST: src = floor(dst * (in / out))."""
    W, H = size
    h, w = img.shape[:2]
    ys = np.minimum((np.arange(H) * (h / H)).astype(np.int64), h - 1)
    xs = np.minimum((np.arange(W) * (w / W)).astype(np.int64), w - 1)
    return img[ys][:, xs]


def resize_bilinear(img: np.ndarray, size: Tuple[int, int]) -> np.ndarray:
    """cv2 INTER_LINEAR (half-pixel centres, clamped)."""
    W, H = size
    h, w = img.shape[:2]

    def coords(n_out, n_in):
        s = (np.arange(n_out) + 0.5) * (n_in / n_out) - 0.5
        s = np.clip(s, 0, n_in - 1)
        i0 = np.floor(s).astype(np.int64)
        i1 = np.minimum(i0 + 1, n_in - 1)
        return i0, i1, s - i0

    y0, y1, ly = coords(H, h)
    x0, x1, lx = coords(W, w)
    x = img.astype(np.float64)
    if x.ndim == 2:
        x = x[..., None]
    top = x[y0][:, x0] * (1 - lx)[None, :, None] + x[y0][:, x1] * lx[None, :, None]
    bot = x[y1][:, x0] * (1 - lx)[None, :, None] + x[y1][:, x1] * lx[None, :, None]
    out = top * (1 - ly)[:, None, None] + bot * ly[:, None, None]
    if img.ndim == 2:
        out = out[..., 0]
    if img.dtype == np.uint8:
        return np.clip(np.rint(out), 0, 255).astype(np.uint8)
    return out.astype(img.dtype)

"""Native baseline-JPEG entropy decode (csrc/jpeg.cpp) + the NumPy oracle of the GPU pixel stage
(data/jpeg.py) against PIL's libjpeg decode -- the decoder behind the reference server's
``cv2.imdecode(IMREAD_COLOR)`` (services/vision_analysis/server.py:117). Bit-exact: both run the
ISLOW IDCT, fancy chroma upsampling and the fixed-point YCbCr -> RGB."""
import io

import numpy as np
import pytest
from PIL import Image

from robotic_discovery_platform_amd.data.image_io import decode_image, encode_jpeg
from robotic_discovery_platform_amd.data.jpeg import coefs_to_rgb_reference, decode_coefs
from robotic_discovery_platform_amd.ops import native

pytestmark = pytest.mark.skipif(native(build_if_missing=False) is None, reason="native extension not built")


def _frame(h, w, seed=0):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = np.stack([(x * 255 // max(w - 1, 1)), (y * 255 // max(h - 1, 1)), ((x + y) * 3) % 256], -1)
    return np.clip(base + rng.integers(-40, 40, (h, w, 3)), 0, 255).astype(np.uint8)


def _jpeg(rgb, **kw):
    buf = io.BytesIO()
    Image.fromarray(rgb, "L" if rgb.ndim == 2 else "RGB").save(buf, format="JPEG", **kw)
    return buf.getvalue()


def _pil(data):
    return np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))


@pytest.mark.parametrize("subsampling", [0, 1, 2])  # PIL: 4:4:4, 4:2:2, 4:2:0
@pytest.mark.parametrize("hw", [(480, 640), (37, 53), (16, 16), (1, 9)])
@pytest.mark.parametrize("restart_rows", [0, 1, 3])
def test_oracle_bit_exact_vs_pil(subsampling, hw, restart_rows):
    rgb = _frame(*hw, seed=hw[0] + subsampling)
    kw = dict(quality=90, subsampling=subsampling)
    if restart_rows:
        kw["restart_marker_rows"] = restart_rows
    data = _jpeg(rgb, **kw)
    jc = decode_coefs(data)
    assert jc is not None and jc.shape == (hw[0], hw[1], 3)
    np.testing.assert_array_equal(coefs_to_rgb_reference(jc), _pil(data))


@pytest.mark.parametrize("quality", [30, 75, 100])
def test_quality_range_and_grayscale(quality):
    rgb = _frame(64, 96, seed=quality)
    data = _jpeg(rgb, quality=quality)
    np.testing.assert_array_equal(coefs_to_rgb_reference(decode_coefs(data)), _pil(data))
    gray = _jpeg(rgb[..., 0].copy(), quality=quality)
    np.testing.assert_array_equal(coefs_to_rgb_reference(decode_coefs(gray)), _pil(gray))


def test_parallel_equals_serial():
    data = encode_jpeg(_frame(480, 640, 3), 95, restart_rows=1)
    a, b = decode_coefs(data, parallel=True), decode_coefs(data, parallel=False)
    assert bool((a.meta == b.meta).all()) and bool((a.coefs == b.coefs).all())
    # the client's encoder output decodes the same through PIL (restart markers are standard baseline)
    np.testing.assert_array_equal(coefs_to_rgb_reference(a), decode_image(data, True, "RGB"))


def test_meta_layout():
    jc = decode_coefs(_jpeg(_frame(48, 80), quality=90, subsampling=2))
    g = jc.geo.numpy()
    assert (g[0], g[1], g[2], g[3], g[4]) == (80, 48, 3, 2, 2)
    # Y: 2x2 sampling over 5 x 3 MCUs of 16 x 16 -> 10 x 6 blocks; chroma 5 x 3 each
    assert list(g[8:12]) == [2, 2, 10, 6] and list(g[16:20]) == [1, 1, 5, 3] and list(g[24:28]) == [1, 1, 5, 3]
    assert jc.blocks == 60 + 15 + 15 == g[5] and jc.coefs.numel() == jc.blocks * 64
    assert jc.qt.numel() == 192 and int(jc.qt.min()) >= 1


def test_unsupported_and_corrupt_streams_return_none():
    rgb = _frame(64, 64)
    assert decode_coefs(_jpeg(rgb, quality=90, progressive=True)) is None  # progressive: PIL path
    assert decode_coefs(b"notajpeg") is None
    data = _jpeg(rgb, quality=90)
    decode_coefs(data[: len(data) // 3])  # truncated scan: no crash
    for cut in (2, 20, 100, 300):
        decode_coefs(data[:cut])  # headers cut anywhere: None or a (zero-filled) decode, never a crash
    rng = np.random.default_rng(1)
    for _ in range(20):  # flipped bytes anywhere
        b = bytearray(data)
        for i in rng.integers(0, len(b), 8):
            b[i] = int(rng.integers(0, 256))
        decode_coefs(bytes(b))


def test_restart_marker_count_mismatch_is_corrupt():
    data = bytearray(encode_jpeg(_frame(64, 64), 90, restart_rows=1))
    i = data.index(b"\xff\xd0")
    data[i + 1] = 0x00  # an RST marker turned into a stuffed byte: one segment short
    assert decode_coefs(bytes(data)) is None


def test_cpu_pipeline_takes_coefficients():
    import torch
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    from robotic_discovery_platform_amd.serve.engine import CpuFramePipeline
    torch.manual_seed(0)
    m = UNetRef(3, 1).eval()
    p = CpuFramePipeline(m, DEFAULT_K, 0.001, H=48, W=64, size=32)
    bgr = _frame(48, 64)
    data = encode_jpeg(bgr, 95, restart_rows=1)
    depth = np.full((48, 64), 500, np.uint16)
    p.submit(decode_coefs(data), depth, rgb=True)
    a = p.collect()
    b = p.process(decode_image(data, True, "BGR"), depth)
    np.testing.assert_array_equal(a.mask, b.mask)


def test_forged_huge_header_is_refused():
    """An SOF claiming 65535 x 65535 (a 25 GB coefficient allocation) is rejected before allocating."""
    data = bytearray(_jpeg(_frame(16, 16), quality=90))
    i = data.index(b"\xff\xc0")
    data[i + 5:i + 9] = b"\xff\xff\xff\xff"  # height, width
    assert decode_coefs(bytes(data)) is None


# ------------------------------------------------------------------ colour space / orientation fallbacks
def _segments(data):
    """(marker, payload-with-length) list up to SOS, and the rest (SOS .. EOI)."""
    p, segs = 2, []
    while True:
        m = data[p + 1]
        ln = (data[p + 2] << 8) | data[p + 3]
        if m == 0xDA:
            return segs, data[p:]
        segs.append((m, data[p + 2:p + 2 + ln]))
        p += 2 + ln


def _assemble(segs, rest):
    return b"\xff\xd8" + b"".join(bytes([0xFF, m]) + pl for m, pl in segs) + rest


def _adobe(transform):
    body = b"Adobe" + bytes([0, 100, 0, 0, 0, 0, transform])
    return (0xEE, bytes([0, len(body) + 2]) + body)


def test_adobe_rgb_jpeg_falls_back_to_libjpeg_semantics():
    """An Adobe APP14 marker with transform 0 (no JFIF) means RGB components: libjpeg -- and the
    reference's cv2.imdecode -- skip the YCbCr conversion, so the native (YCbCr) path must decline."""
    segs, rest = _segments(_jpeg(_frame(48, 64, 3), quality=92, subsampling=0))
    segs = [s for s in segs if s[0] != 0xE0]  # drop JFIF
    for transform, native_ok in ((0, False), (1, True)):
        data = _assemble([_adobe(transform)] + segs, rest)
        jc = decode_coefs(data, parallel=False)
        assert (jc is not None) == native_ok
        want = _pil(data)
        assert np.array_equal(decode_image(data, True, "RGB"), want)
        if native_ok:
            assert np.array_equal(coefs_to_rgb_reference(jc), want)


def test_rgb_component_ids_fall_back():
    """No JFIF / Adobe marker and component ids 'R', 'G', 'B': libjpeg decodes without conversion."""
    segs, rest = _segments(_jpeg(_frame(40, 56, 4), quality=92, subsampling=0))
    segs = [s for s in segs if s[0] != 0xE0]
    out = []
    for m, pl in segs:
        if m in (0xC0, 0xC1):
            pl = bytearray(pl)
            for c in range(3):
                pl[2 + 6 + 3 * c] = b"RGB"[c]
            pl = bytes(pl)
        out.append((m, pl))
    rest = bytearray(rest)  # SOS: ff da len(2) ns (id, tables) x 3
    for k in range(3):
        rest[5 + 2 * k] = b"RGB"[k]
    data = _assemble(out, bytes(rest))
    assert decode_coefs(data, parallel=False) is None
    assert np.array_equal(decode_image(data, True, "RGB"), _pil(data))


def test_exif_rotated_jpeg_is_transposed_like_cv2():
    """cv2.imdecode(IMREAD_COLOR) applies the EXIF orientation: the native path declines such streams
    and the fallback rotates (orientation 6: 90 degrees clockwise)."""
    rgb = _frame(24, 40, 5)
    ex = Image.Exif()
    ex[0x0112] = 6
    buf = io.BytesIO()
    Image.fromarray(rgb, "RGB").save(buf, format="JPEG", quality=95, exif=ex.tobytes())
    data = buf.getvalue()
    assert decode_coefs(data, parallel=False) is None
    out = decode_image(data, True, "RGB")
    assert out.shape == (40, 24, 3)
    assert np.array_equal(out, np.rot90(_pil(data), k=-1))
    ex[0x0112] = 1  # upright EXIF: the native path takes it
    buf = io.BytesIO()
    Image.fromarray(rgb, "RGB").save(buf, format="JPEG", quality=95, exif=ex.tobytes())
    assert decode_coefs(buf.getvalue(), parallel=False) is not None

"""Native grayscale PNG codec (csrc/codecs.cpp): plain and banded streams against PIL, the band index's
fallbacks, and hostile inputs. The reference's per-frame codecs are cv2.imencode / imdecode of the
16-bit depth PNG and the mask PNG (client.py:67, server.py:118,142)."""
import io
import struct
import zlib

import numpy as np
import pytest
from PIL import Image

from robotic_discovery_platform_amd.data.image_io import decode_image, encode_png
from robotic_discovery_platform_amd.ops import native

C = native(build_if_missing=False)
pytestmark = pytest.mark.skipif(C is None, reason="native extension not built")


def _chunks(data):
    p, out = 8, []
    while p < len(data):
        n = struct.unpack(">I", data[p:p + 4])[0]
        out.append((data[p + 4:p + 8], p, n))
        p += 12 + n
    return out


def _rechunk(data, ctype, payload):
    """Replace the payload of chunk `ctype` (CRC recomputed)."""
    for t, p, n in _chunks(data):
        if t == ctype:
            body = ctype + payload
            return data[:p] + struct.pack(">I", len(payload)) + body + struct.pack(">I", zlib.crc32(body)) + \
                data[p + 12 + n:]
    raise KeyError(ctype)


def _img(h, w, dtype, seed=0):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    if dtype == np.uint16:
        return ((x * 37 + y * 11) % 4000 + rng.integers(0, 3, (h, w)) + 300).astype(np.uint16)
    return (((x // 7 + y // 5) % 2) * 255).astype(np.uint8)


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16])
@pytest.mark.parametrize("hw", [(480, 640), (1, 17), (17, 1), (3, 5), (100, 33)])
@pytest.mark.parametrize("bands", [1, 2, 4, 8, 64])
def test_roundtrip_and_pil_agree(dtype, hw, bands):
    a = _img(*hw, dtype, seed=hw[0])
    data = encode_png(a, compress_level=1, bands=bands)
    types = [t for t, _, _ in _chunks(data)]
    assert (b"rdPs" in types) == (min(bands, hw[0]) > 1)
    pil = np.asarray(Image.open(io.BytesIO(data)))
    np.testing.assert_array_equal(pil.astype(a.dtype), a)  # an ordinary PNG for other readers
    for par in (True, False):
        t = C.png_decode(data, par).numpy()
        np.testing.assert_array_equal(t.view(np.uint16) if dtype == np.uint16 else t, a)
    out = decode_image(data, color=False)
    assert out.dtype == a.dtype
    np.testing.assert_array_equal(out, a)


def test_banded_path_is_taken():
    """Our banded files decode through the parallel band path (mode 2: banded only). A broken zlib
    header (or a preset-dictionary flag) is rejected there too, as libpng rejects it."""
    a = _img(480, 640, np.uint16)
    data = encode_png(a, 1, bands=8)
    np.testing.assert_array_equal(C.png_decode(data, 2).numpy().view(np.uint16), a)
    for t, p, n in _chunks(data):
        if t == b"IDAT":
            z = bytearray(data[p + 8:p + 8 + n])
    for flip in (0x1F, 0x20):  # check bits wrong / FDICT set
        zb = bytearray(z)
        zb[1] ^= flip
        bad = _rechunk(data, b"IDAT", bytes(zb))
        assert C.png_decode(bad, 0) is None and C.png_decode(bad, 2) is None and C.png_decode(bad, 1) is None


def test_banded_band_input_fully_consumed():
    """Every band's compressed bytes must be consumed: a band index whose first band stops short of the
    data (rows full early) is not taken, and the serial decode stays authoritative."""
    a = _img(256, 320, np.uint16)
    data = encode_png(a, 1, bands=4)
    for t, p, n in _chunks(data):
        if t == b"rdPs":
            idx = bytearray(data[p + 8:p + 8 + n])
    # move band 1's start one byte later: band 0 keeps a trailing byte it never decodes
    off = int.from_bytes(idx[20:24], "big")
    idx[20:24] = (off + 1).to_bytes(4, "big")
    bad = _rechunk(data, b"rdPs", bytes(idx))
    assert C.png_decode(bad, 2) is None


def test_bad_index_falls_back_to_serial():
    a = _img(120, 64, np.uint16)
    data = encode_png(a, 1, bands=4)
    idx = bytearray([c for t, p, n in _chunks(data) if t == b"rdPs" for c in data[p + 8:p + 8 + n]])
    cases = []
    wrong_off = bytearray(idx)
    wrong_off[8 + 8 * 2 + 7] ^= 0x01  # band 2 offset off by one
    cases.append(_rechunk(data, b"rdPs", bytes(wrong_off)))
    wrong_row = bytearray(idx)
    wrong_row[8 + 8 * 1 + 3] ^= 0x02  # band 1 first row moved
    cases.append(_rechunk(data, b"rdPs", bytes(wrong_row)))
    cases.append(_rechunk(data, b"rdPs", bytes(idx[:12])))  # truncated index
    bad_crc = bytearray(data)
    p = [p for t, p, n in _chunks(data) if t == b"rdPs"][0]
    bad_crc[p + 8 + 9] ^= 0xFF  # payload changed, CRC not: index ignored
    cases.append(bytes(bad_crc))
    for c in cases:
        np.testing.assert_array_equal(C.png_decode(c, True).numpy().view(np.uint16), a)


def test_hostile_inputs_never_crash():
    a = _img(64, 64, np.uint16)
    data = encode_png(a, 1, bands=4)
    rng = np.random.default_rng(0)
    for cut in range(8, len(data), max(1, len(data) // 40)):
        C.png_decode(data[:cut], True)  # truncated anywhere
    for _ in range(200):
        b = bytearray(data)
        for i in rng.integers(8, len(b), 4):
            b[i] = int(rng.integers(0, 256))
        r = C.png_decode(bytes(b), True)
        assert r is None or tuple(r.shape) == (64, 64) or r.dim() == 2
    # an index claiming thousands of bands / huge offsets
    idx = struct.pack(">BxxxI", 1, 4000) + b"".join(struct.pack(">II", i, 2 + i) for i in range(4000))
    forged = _rechunk(data, b"rdPs", idx)
    np.testing.assert_array_equal(C.png_decode(forged, True).numpy().view(np.uint16), a)


def test_encoder_rejects_bad_arguments():
    with pytest.raises(Exception):
        C.png_encode(__import__("torch").zeros(4, 4, dtype=__import__("torch").float32), 1, 1)

// Native PNG codec for the serving hot path (zlib), callable with the Python GIL released.
//
// The reference decodes the client's 16-bit depth PNG with cv2.imdecode(IMREAD_UNCHANGED) and
// encodes the response mask with cv2.imencode('.png') per frame (services/vision_analysis/
// server.py:118,142); its client encodes the depth frame with cv2.imencode('.png') (client.py:67).
// Without OpenCV, PIL does both, but its PNG reader walks the IDAT chunks in Python, so a server
// thread holds the GIL for most of a 640x480 depth decode and concurrent streams serialise on it.
// This reader/writer does the whole job in C++:
//   decode: non-interlaced grayscale 8 / 16 bit (IHDR colour type 0) -> u8 or native-endian u16;
//           chunk walk, IDAT concatenation, inflate, the five scanline filters. Anything else
//           (colour, palette, interlaced) returns "unsupported" and the caller uses PIL.
//   encode: grayscale 8 / 16 bit, filter type 0 per row, deflate at the given level, CRC'd chunks.
//
// Banded streams. One inflate of a 640x480x16-bit frame is ~2 ms of serial work on the request's
// critical path. The encoder can split the rows into bands, each deflated from a fresh dictionary and
// ended byte-aligned without the final bit (a sync flush), so the IDAT data is still ONE ordinary
// zlib stream that every PNG reader decodes. A private ancillary chunk `rdPs` (ignored by other
// readers: lower-case first letter = ancillary, second = private) before IDAT records each band's
// first row and its offset in the zlib stream; this decoder inflates (and unfilters) the bands in
// parallel on the shared host pool, checks the stream's Adler-32 from the bands' checksums, and falls
// back to the serial path whenever the index does not describe the stream exactly.
#include <zlib.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "host_pool.h"

namespace {
template <class F>
void host_pool_for(int n, F&& f) { rdp::host_pool().parallel_for(n, std::function<void(int)>(f)); }
}  // namespace

namespace {

inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
inline void put32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back(x >> 24); v.push_back(x >> 16); v.push_back(x >> 8); v.push_back(x);
}
const uint8_t kSig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
const uint64_t kMaxPixels = 89478485;  // PIL Image.MAX_IMAGE_PIXELS

struct Hdr {
  uint32_t w = 0, h = 0;
  int bd = 0, ct = 0, interlace = 0;
};

// -1 not a PNG / truncated, -2 unsupported format
int parse_header(const uint8_t* d, long n, Hdr& hd) {
  if (n < 33 || std::memcmp(d, kSig, 8) != 0) return -1;
  if (be32(d + 8) != 13 || std::memcmp(d + 12, "IHDR", 4) != 0) return -1;
  hd.w = be32(d + 16);
  hd.h = be32(d + 20);
  hd.bd = d[24];
  hd.ct = d[25];
  hd.interlace = d[28];
  if (hd.w == 0 || hd.h == 0 || hd.w > (1u << 16) || hd.h > (1u << 16)) return -1;
  if (hd.ct != 0 || (hd.bd != 8 && hd.bd != 16) || hd.interlace != 0 || d[26] != 0 || d[27] != 0) return -2;
  // The size comes from an untrusted request: refuse it before anything is allocated from it.
  // (a) PIL's decompression-bomb limit (Image.MAX_IMAGE_PIXELS), the bound of the reader this replaces;
  // (b) the filtered scanlines cannot be larger than deflate can expand the whole file to (at most
  //     1032:1), so a header-only "image" of a few dozen bytes cannot claim gigabytes.
  const uint64_t px = (uint64_t)hd.w * hd.h;
  const uint64_t raw = ((uint64_t)hd.w * (hd.bd / 8) + 1) * hd.h;
  if (px > kMaxPixels || raw > (uint64_t)n * 1032u) return -1;
  return 0;
}

inline uint8_t paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  return (uint8_t)((pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c));
}

// Unfilter rows [y0, y1) of `raw` (stride + 1 bytes per row, filter byte first) into out (native-endian
// samples). `prev`: the reconstructed previous row (filtered bytes' order, i.e. big-endian), or null
// for "row y0 - 1 is all zero" (y0 == 0, or a band that starts with a filter not referencing it).
bool unfilter(const uint8_t* raw, size_t stride, int bpp, uint32_t y0, uint32_t y1, const uint8_t* prev_in,
              uint8_t* out, uint8_t* last_row_out) {
  std::vector<uint8_t> prev(stride, 0), cur(stride);
  if (prev_in) std::memcpy(prev.data(), prev_in, stride);
  for (uint32_t y = y0; y < y1; ++y) {
    const uint8_t f = raw[y * (stride + 1)];
    const uint8_t* s = raw + y * (stride + 1) + 1;
    switch (f) {
      case 0: std::memcpy(cur.data(), s, stride); break;
      case 1:
        for (size_t i = 0; i < stride; ++i) cur[i] = s[i] + (i >= (size_t)bpp ? cur[i - bpp] : 0);
        break;
      case 2:
        for (size_t i = 0; i < stride; ++i) cur[i] = s[i] + prev[i];
        break;
      case 3:
        for (size_t i = 0; i < stride; ++i)
          cur[i] = s[i] + (uint8_t)(((i >= (size_t)bpp ? cur[i - bpp] : 0) + prev[i]) >> 1);
        break;
      case 4:
        for (size_t i = 0; i < stride; ++i) {
          const int a = i >= (size_t)bpp ? cur[i - bpp] : 0, c = i >= (size_t)bpp ? prev[i - bpp] : 0;
          cur[i] = s[i] + paeth(a, prev[i], c);
        }
        break;
      default: return false;
    }
    uint8_t* o = out + (size_t)y * stride;
    if (bpp == 2) {  // big-endian samples -> native (little-endian)
      for (size_t i = 0; i < stride; i += 2) { o[i] = cur[i + 1]; o[i + 1] = cur[i]; }
    } else {
      std::memcpy(o, cur.data(), stride);
    }
    prev.swap(cur);
  }
  if (last_row_out) std::memcpy(last_row_out, prev.data(), stride);
  return true;
}

struct Band {
  uint32_t row0;
  uint32_t zoff;  // offset of the band's deflate data in the zlib stream (band 0: 2, after the header)
};

// The rdPs index: u8 version (1), 3 reserved bytes, u32 band count, then per band u32 first row and
// u32 zlib-stream offset (all big-endian). Structurally validated here; checked against the stream
// while inflating.
bool parse_index(const uint8_t* c, uint32_t len, uint32_t h, size_t zlen, std::vector<Band>& bands) {
  if (len < 8 || c[0] != 1) return false;
  const uint32_t nb = be32(c + 4);
  if (nb < 2 || nb > h || nb > 4096 || len != 8 + 8 * nb) return false;
  bands.resize(nb);
  for (uint32_t k = 0; k < nb; ++k) {
    bands[k].row0 = be32(c + 8 + 8 * k);
    bands[k].zoff = be32(c + 12 + 8 * k);
    if (k == 0 ? (bands[k].row0 != 0 || bands[k].zoff != 2)
               : (bands[k].row0 <= bands[k - 1].row0 || bands[k].zoff <= bands[k - 1].zoff))
      return false;
  }
  return bands.back().row0 < h && bands.back().zoff + 4 < zlen;
}

// inflate raw-deflate `in` into exactly `out_len` bytes; `final`: the data must end the stream
bool inflate_band(const uint8_t* in, size_t in_len, uint8_t* out, size_t out_len, bool final) {
  z_stream zs;
  std::memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, -15) != Z_OK) return false;
  zs.next_in = const_cast<uint8_t*>(in);
  zs.avail_in = (uInt)in_len;
  zs.next_out = out;
  zs.avail_out = (uInt)out_len;
  const int zr = inflate(&zs, final ? Z_FINISH : Z_SYNC_FLUSH);
  bool ok = zs.avail_out == 0 && (final ? zr == Z_STREAM_END : (zr == Z_OK || zr == Z_BUF_ERROR ||
                                                                 zr == Z_STREAM_END));
  const bool ended = zr == Z_STREAM_END;
  if (ok && !final && zs.avail_in > 0) {
    // the band's rows are full: what is left of its input (the flush's empty stored block) must
    // decode to nothing -- input that would produce more bytes belongs to no row
    uint8_t spare = 0;
    zs.next_out = &spare;
    zs.avail_out = 1;
    const int z2 = inflate(&zs, Z_SYNC_FLUSH);
    ok = zs.avail_out == 1 && (z2 == Z_OK || z2 == Z_BUF_ERROR);
  }
  // every byte of the band's input consumed, as the serial decoder (libpng / cv2) would read it
  ok = ok && zs.avail_in == 0;
  inflateEnd(&zs);
  return ok && (final || !ended);  // a non-final band must not carry the final block
}

// the zlib stream header (RFC 1950): deflate, window <= 32 KiB, valid check bits, no preset dictionary
bool zlib_header_ok(const std::vector<uint8_t>& z) {
  if (z.size() < 6) return false;
  const unsigned cmf = z[0], flg = z[1];
  return (cmf & 15) == 8 && (cmf >> 4) <= 7 && ((cmf << 8) | flg) % 31 == 0 && !(flg & 0x20);
}

// parallel decode along the rdPs index; false: fall back to the serial decoder
bool decode_banded(const std::vector<uint8_t>& z, const std::vector<Band>& bands, const Hdr& hd, int bpp,
                   size_t stride, uint8_t* out) {
  const size_t nb = bands.size();
  const size_t zdata_end = z.size() - 4;  // Adler-32 trailer
  std::vector<uint8_t> raw((stride + 1) * hd.h);
  std::vector<uLong> adl(nb);
  std::vector<char> ok(nb, 0);
  auto row_end = [&](size_t k) { return k + 1 < nb ? bands[k + 1].row0 : hd.h; };
  host_pool_for((int)nb, [&](int k) {
    const size_t r0 = bands[k].row0, r1 = row_end(k);
    const size_t z0 = bands[k].zoff, z1 = k + 1 < nb ? bands[k + 1].zoff : zdata_end;
    if (z1 <= z0 || z1 > zdata_end) return;
    uint8_t* dst = raw.data() + r0 * (stride + 1);
    const size_t len = (r1 - r0) * (stride + 1);
    if (!inflate_band(z.data() + z0, z1 - z0, dst, len, (size_t)k + 1 == nb)) return;
    adl[k] = adler32(adler32(0L, Z_NULL, 0), dst, (uInt)len);
    ok[k] = 1;
  });
  uLong a = adler32(0L, Z_NULL, 0);
  for (size_t k = 0; k < nb; ++k) {
    if (!ok[k]) return false;
    a = adler32_combine(a, adl[k], (z_off_t)((row_end(k) - bands[k].row0) * (stride + 1)));
  }
  if (a != be32(z.data() + zdata_end)) return false;
  // unfilter: bands whose first row does not reference the row above are independent
  bool indep = true;
  for (size_t k = 1; k < nb; ++k) {
    const uint8_t f = raw[(size_t)bands[k].row0 * (stride + 1)];
    indep &= f == 0 || f == 1;
  }
  if (indep) {
    std::vector<char> uok(nb, 0);
    host_pool_for((int)nb, [&](int k) {
      uok[k] = unfilter(raw.data(), stride, bpp, bands[k].row0, row_end(k), nullptr, out, nullptr);
    });
    for (char u : uok)
      if (!u) return false;
    return true;
  }
  return unfilter(raw.data(), stride, bpp, 0, hd.h, nullptr, out, nullptr);
}

void put_chunk(std::vector<uint8_t>& v, const char* type, const uint8_t* data, size_t len) {
  put32(v, (uint32_t)len);
  const size_t t0 = v.size();
  v.insert(v.end(), type, type + 4);
  if (len) v.insert(v.end(), data, data + len);
  put32(v, (uint32_t)crc32(0L, v.data() + t0, (uInt)(len + 4)));
}

}  // namespace

extern "C" {

// width, height, bit depth of a supported PNG; returns 0, -1 (not PNG / corrupt) or -2 (unsupported)
int rdp_png_info(const uint8_t* d, long n, int* w, int* h, int* bd) {
  Hdr hd;
  const int r = parse_header(d, n, hd);
  if (r) return r;
  *w = (int)hd.w;
  *h = (int)hd.h;
  *bd = hd.bd;
  return 0;
}

// decode into out (h * w * bd/8 bytes; 16-bit samples native-endian). 0 ok, -1 corrupt, -2 unsupported.
// `parallel`: use an rdPs band index if the file has one.
int rdp_png_decode(const uint8_t* d, long n, uint8_t* out, long out_bytes, int parallel) {
  Hdr hd;
  int r = parse_header(d, n, hd);
  if (r) return r;
  const int bpp = hd.bd / 8;  // grayscale: bytes per pixel
  const size_t stride = (size_t)hd.w * bpp;
  if ((long)(stride * hd.h) > out_bytes) return -1;
  // concatenate IDAT payloads; remember an rdPs index seen before the first IDAT
  std::vector<uint8_t> z;
  long p = 8, idx = -1;
  uint32_t idx_len = 0;
  bool end = false;
  while (p + 12 <= n) {
    const uint32_t len = be32(d + p);
    const uint8_t* type = d + p + 4;
    if ((long)len > n - p - 12) return -1;
    if (std::memcmp(type, "IDAT", 4) == 0) z.insert(z.end(), d + p + 8, d + p + 8 + len);
    if (std::memcmp(type, "rdPs", 4) == 0 && z.empty() && idx < 0 &&
        be32(d + p + 8 + len) == (uint32_t)crc32(0L, d + p + 4, len + 4)) {
      idx = p + 8;
      idx_len = len;
    }
    if (std::memcmp(type, "IEND", 4) == 0) { end = true; break; }
    p += 12 + (long)len;
  }
  if (!end && z.empty()) return -1;
  std::vector<Band> bands;
  if (parallel && idx >= 0 && zlib_header_ok(z) && parse_index(d + idx, idx_len, hd.h, z.size(), bands) &&
      decode_banded(z, bands, hd, bpp, stride, out))
    return 0;
  if (parallel == 2) return -3;  // banded path only (tests): not taken
  const size_t raw_len = (stride + 1) * hd.h;
  std::vector<uint8_t> raw(raw_len);
  z_stream zs;
  std::memset(&zs, 0, sizeof(zs));
  if (inflateInit(&zs) != Z_OK) return -1;
  zs.next_in = z.data();
  zs.avail_in = (uInt)z.size();
  zs.next_out = raw.data();
  zs.avail_out = (uInt)raw_len;
  const int zr = inflate(&zs, Z_FINISH);
  const size_t got = raw_len - zs.avail_out;
  inflateEnd(&zs);
  if ((zr != Z_STREAM_END && zr != Z_OK && zr != Z_BUF_ERROR) || got != raw_len) return -1;
  return unfilter(raw.data(), stride, bpp, 0, hd.h, nullptr, out, nullptr) ? 0 : -1;
}

// Grayscale PNG of img (h x w, row-major; bpp 1 = u8, 2 = native-endian u16), filter type 0 per row,
// deflated at `level` in `bands` row bands (> 1: the banded stream + rdPs index described above, the
// bands compressed in parallel). Returns the encoded size, or -1 if cap is too small / zlib failed.
long rdp_png_encode_gray(const uint8_t* img, int w, int h, int bpp, int level, int bands, uint8_t* out, long cap) {
  if (w <= 0 || h <= 0 || (bpp != 1 && bpp != 2)) return -1;
  const size_t stride = (size_t)w * bpp;
  const int nb = std::max(1, std::min(bands, h));
  std::vector<std::vector<uint8_t>> zb(nb);
  std::vector<uLong> adl(nb);
  std::vector<char> ok(nb, 0);
  auto row0 = [&](int k) { return (int)((long)h * k / nb); };
  host_pool_for(nb, [&](int k) {
    const int r0 = row0(k), r1 = row0(k + 1);
    std::vector<uint8_t> raw((stride + 1) * (r1 - r0));
    for (int y = r0; y < r1; ++y) {
      uint8_t* o = raw.data() + (size_t)(y - r0) * (stride + 1);
      o[0] = 0;
      const uint8_t* s = img + (size_t)y * stride;
      if (bpp == 2) {  // native -> big-endian samples
        for (size_t i = 0; i < stride; i += 2) { o[1 + i] = s[i + 1]; o[2 + i] = s[i]; }
      } else {
        std::memcpy(o + 1, s, stride);
      }
    }
    adl[k] = adler32(adler32(0L, Z_NULL, 0), raw.data(), (uInt)raw.size());
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return;
    std::vector<uint8_t>& zo = zb[k];
    zo.resize(deflateBound(&zs, raw.size()) + 16);
    zs.next_in = raw.data();
    zs.avail_in = (uInt)raw.size();
    zs.next_out = zo.data();
    zs.avail_out = (uInt)zo.size();
    const bool last = k + 1 == nb;
    const int zr = deflate(&zs, last ? Z_FINISH : Z_SYNC_FLUSH);
    const bool good = last ? zr == Z_STREAM_END : (zr == Z_OK && zs.avail_in == 0 && zs.avail_out > 0);
    zo.resize(zo.size() - zs.avail_out);
    deflateEnd(&zs);
    ok[k] = good;
  });
  std::vector<uint8_t> z = {0x78, 0x01};  // zlib header: deflate, 32K window (FLEVEL is advisory)
  std::vector<uint8_t> index(8 + 8 * nb, 0);
  index[0] = 1;
  uLong a = adler32(0L, Z_NULL, 0);
  for (int k = 0; k < nb; ++k) {
    if (!ok[k]) return -1;
    const uint32_t r0 = row0(k), zo = (uint32_t)z.size();
    uint8_t* e = index.data() + 8 + 8 * k;
    e[0] = r0 >> 24; e[1] = r0 >> 16; e[2] = r0 >> 8; e[3] = r0;
    e[4] = zo >> 24; e[5] = zo >> 16; e[6] = zo >> 8; e[7] = zo;
    z.insert(z.end(), zb[k].begin(), zb[k].end());
    a = adler32_combine(a, adl[k], (z_off_t)((row0(k + 1) - row0(k)) * (stride + 1)));
  }
  put32(z, (uint32_t)a);
  index[4] = (uint8_t)(nb >> 24); index[5] = (uint8_t)(nb >> 16); index[6] = (uint8_t)(nb >> 8); index[7] = (uint8_t)nb;
  std::vector<uint8_t> v(kSig, kSig + 8);
  uint8_t ihdr[13];
  const uint32_t W = w, H = h;
  ihdr[0] = W >> 24; ihdr[1] = W >> 16; ihdr[2] = W >> 8; ihdr[3] = W;
  ihdr[4] = H >> 24; ihdr[5] = H >> 16; ihdr[6] = H >> 8; ihdr[7] = H;
  ihdr[8] = (uint8_t)(8 * bpp); ihdr[9] = 0; ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
  put_chunk(v, "IHDR", ihdr, 13);
  if (nb > 1) put_chunk(v, "rdPs", index.data(), index.size());
  put_chunk(v, "IDAT", z.data(), z.size());
  put_chunk(v, "IEND", nullptr, 0);
  if ((long)v.size() > cap) return -1;
  std::memcpy(out, v.data(), v.size());
  return (long)v.size();
}

long rdp_png_encode_bound(int w, int h, int bpp, int bands) {
  const uLong raw = (uLong)((size_t)w * bpp + 1) * h;
  return (long)compressBound(raw) + 64L * std::max(1, bands) + 128;
}

}  // extern "C"

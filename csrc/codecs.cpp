// Native PNG codec for the serving hot path (zlib), callable with the Python GIL released.
//
// The reference decodes the client's 16-bit depth PNG with cv2.imdecode(IMREAD_UNCHANGED) and
// encodes the response mask with cv2.imencode('.png') per frame (services/vision_analysis/
// server.py:118,142). Without OpenCV, PIL does both, but its PNG reader walks the IDAT chunks in
// Python, so a server thread holds the GIL for most of a 640x480 depth decode and concurrent streams
// serialise on it. This reader/writer does the whole job in C++:
//   decode: non-interlaced grayscale 8 / 16 bit (IHDR colour type 0) -> u8 or native-endian u16;
//           chunk walk, IDAT concatenation, one inflate, the five scanline filters. Anything else
//           (colour, palette, interlaced) returns "unsupported" and the caller uses PIL.
//   encode: 8-bit grayscale, filter type 0 per row, deflate at the given level, CRC'd chunks.
#include <zlib.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

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

// decode into out (h * w * bd/8 bytes; 16-bit samples native-endian). 0 ok, -1 corrupt, -2 unsupported
int rdp_png_decode(const uint8_t* d, long n, uint8_t* out, long out_bytes) {
  Hdr hd;
  int r = parse_header(d, n, hd);
  if (r) return r;
  const int bpp = hd.bd / 8;  // grayscale: bytes per pixel
  const size_t stride = (size_t)hd.w * bpp;
  if ((long)(stride * hd.h) > out_bytes) return -1;
  // concatenate IDAT payloads
  std::vector<uint8_t> z;
  long p = 8;
  bool end = false;
  while (p + 12 <= n) {
    const uint32_t len = be32(d + p);
    const uint8_t* type = d + p + 4;
    if ((long)len > n - p - 12) return -1;
    if (std::memcmp(type, "IDAT", 4) == 0) z.insert(z.end(), d + p + 8, d + p + 8 + len);
    if (std::memcmp(type, "IEND", 4) == 0) { end = true; break; }
    p += 12 + (long)len;
  }
  if (!end && z.empty()) return -1;
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
  // unfilter in place, row by row (previous row = already reconstructed output row)
  std::vector<uint8_t> prev(stride, 0), cur(stride);
  for (uint32_t y = 0; y < hd.h; ++y) {
    const uint8_t f = raw[y * (stride + 1)];
    const uint8_t* s = raw.data() + y * (stride + 1) + 1;
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
      default: return -1;
    }
    uint8_t* o = out + (size_t)y * stride;
    if (bpp == 2) {  // big-endian samples -> native (little-endian)
      for (size_t i = 0; i < stride; i += 2) { o[i] = cur[i + 1]; o[i + 1] = cur[i]; }
    } else {
      std::memcpy(o, cur.data(), stride);
    }
    prev.swap(cur);
  }
  return 0;
}

// 8-bit grayscale PNG of img (h x w, row-major); returns the encoded size, or -1 if cap is too small
long rdp_png_encode_gray8(const uint8_t* img, int w, int h, int level, uint8_t* out, long cap) {
  std::vector<uint8_t> raw((size_t)(w + 1) * h);
  for (int y = 0; y < h; ++y) {
    raw[(size_t)y * (w + 1)] = 0;
    std::memcpy(&raw[(size_t)y * (w + 1) + 1], img + (size_t)y * w, w);
  }
  uLongf zcap = compressBound(raw.size());
  std::vector<uint8_t> z(zcap);
  if (compress2(z.data(), &zcap, raw.data(), raw.size(), level) != Z_OK) return -1;
  std::vector<uint8_t> v(kSig, kSig + 8);
  auto chunk = [&](const char* type, const uint8_t* data, size_t len) {
    put32(v, (uint32_t)len);
    const size_t t0 = v.size();
    v.insert(v.end(), type, type + 4);
    if (len) v.insert(v.end(), data, data + len);
    put32(v, (uint32_t)crc32(0L, v.data() + t0, (uInt)(len + 4)));
  };
  uint8_t ihdr[13];
  const uint32_t W = w, H = h;
  ihdr[0] = W >> 24; ihdr[1] = W >> 16; ihdr[2] = W >> 8; ihdr[3] = W;
  ihdr[4] = H >> 24; ihdr[5] = H >> 16; ihdr[6] = H >> 8; ihdr[7] = H;
  ihdr[8] = 8; ihdr[9] = 0; ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
  chunk("IHDR", ihdr, 13);
  chunk("IDAT", z.data(), zcap);
  chunk("IEND", nullptr, 0);
  if ((long)v.size() > cap) return -1;
  std::memcpy(out, v.data(), v.size());
  return (long)v.size();
}

long rdp_png_encode_bound(int w, int h) { return (long)compressBound((uLong)(w + 1) * h) + 64; }

}  // extern "C"

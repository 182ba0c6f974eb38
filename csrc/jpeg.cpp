// Baseline JPEG entropy decoder for the serving hot path: Huffman-decodes the scan into quantized DCT
// coefficient planes (int16, natural order), with restart-interval segments decoded in parallel on a
// small native thread pool. The pixel work -- dequantisation, the 8x8 inverse DCT, chroma upsampling
// and YCbCr -> RGB -- runs on the GPU (csrc/serve_kernels.hip, inside the per-frame graph).
//
// Reference: the server decodes the client's colour JPEG with cv2.imdecode(IMREAD_COLOR)
// (/root/reference/services/vision_analysis/server.py:117), i.e. libjpeg(-turbo) with its defaults
// (ISLOW integer IDCT, "fancy" triangle upsampling, fixed-point YCbCr -> RGB); the GPU kernels follow
// those definitions so the decoded frame is the one the reference server would analyse.
//
// Supported: baseline / extended-sequential Huffman (SOF0 / SOF1), 8-bit samples, 1 or 3 components
// in one interleaved scan, sampling factors 1..2, any restart interval. Anything else (progressive,
// arithmetic, 12-bit, non-interleaved multi-scan, CMYK, 4:1:1, ...) reports "unsupported" and the caller
// falls back to PIL. Every read is bounds-checked: a corrupt stream yields an error, never a read past
// the buffer.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <vector>

#include "host_pool.h"

namespace {

constexpr int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
  bool present = false;
  uint8_t bits[17] = {0};
  uint8_t vals[256] = {0};
  // canonical decode: maxcode[l] (-1 none), valptr[l], mincode[l]
  int32_t maxcode[18], valptr[17], mincode[17];
  // 9-bit lookahead: (length << 8) | value, 0 = not in the table
  uint16_t look[512];
  // AC fast path (stb_image style): code + magnitude bits within the 9-bit lookahead decoded in one
  // lookup: (value << 8) | (run << 4) | total bits, 0 = use the slow path
  int16_t fast_ac[512];
  bool build() {
    int code = 0, k = 0;
    int huffcode[257];
    uint8_t huffsize[257];
    for (int l = 1; l <= 16; ++l)
      for (int i = 0; i < bits[l]; ++i) {
        if (k >= 256) return false;
        huffsize[k++] = (uint8_t)l;
      }
    const int n = k;
    k = 0;
    int si = n ? huffsize[0] : 0;
    while (k < n) {
      while (k < n && huffsize[k] == si) huffcode[k++] = code++;
      if (code > (1 << si)) return false;
      code <<= 1;
      ++si;
    }
    int p = 0;
    for (int l = 1; l <= 16; ++l) {
      if (bits[l]) {
        valptr[l] = p;
        mincode[l] = huffcode[p];
        p += bits[l];
        maxcode[l] = huffcode[p - 1];
      } else {
        maxcode[l] = -1;
      }
    }
    maxcode[17] = 0x7fffffff;
    std::memset(look, 0, sizeof(look));
    p = 0;
    for (int l = 1; l <= 9; ++l)
      for (int i = 0; i < bits[l]; ++i, ++p) {
        const int lookbits = huffcode[p] << (9 - l);
        for (int c = 0; c < (1 << (9 - l)); ++c) look[lookbits + c] = (uint16_t)((l << 8) | vals[p]);
      }
    for (int i = 0; i < 512; ++i) {
      fast_ac[i] = 0;
      const uint16_t e = look[i];
      if (!e) continue;
      const int l = e >> 8, rs = e & 0xFF, run = rs >> 4, sz = rs & 15;
      if (sz == 0 || sz > 7 || l + sz > 9) continue;
      const int v = (i >> (9 - l - sz)) & ((1 << sz) - 1);
      const int val = v < (1 << (sz - 1)) ? v - (1 << sz) + 1 : v;
      fast_ac[i] = (int16_t)(val * 256 + run * 16 + l + sz);
    }
    present = true;
    return true;
  }
};

struct Comp {
  int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
  int bw = 0, bh = 0;   // blocks per line / column in the plane (MCU padded)
  long plane_off = 0;   // first coefficient of the plane in the output
};

struct Jpeg {
  int width = 0, height = 0, ncomp = 0, hmax = 1, vmax = 1;
  int mcux = 0, mcuy = 0;  // MCUs per line / column
  int restart = 0;
  Comp comp[3];
  uint16_t qt[4][64];
  bool qt_present[4] = {false, false, false, false};
  Huff dc[4], ac[4];
  long scan_begin = 0, scan_end = 0;  // entropy-coded data [begin, end)
  long total_coefs = 0;
};

inline int be16(const uint8_t* p) { return (p[0] << 8) | p[1]; }

// EXIF orientation (TIFF tag 0x0112 of IFD0) of an APP1 payload; 1 (upright) when absent / unreadable
int exif_orientation(const uint8_t* s, int sl) {
  if (sl < 14 || std::memcmp(s, "Exif\0\0", 6) != 0) return 1;
  const uint8_t* t = s + 6;
  const long tl = sl - 6;
  const bool le = t[0] == 'I' && t[1] == 'I';
  if (!le && !(t[0] == 'M' && t[1] == 'M')) return 1;
  auto u16 = [&](long o) { return le ? (t[o] | (t[o + 1] << 8)) : ((t[o] << 8) | t[o + 1]); };
  auto u32 = [&](long o) {
    return le ? ((uint32_t)t[o] | ((uint32_t)t[o + 1] << 8) | ((uint32_t)t[o + 2] << 16) | ((uint32_t)t[o + 3] << 24))
              : (((uint32_t)t[o] << 24) | ((uint32_t)t[o + 1] << 16) | ((uint32_t)t[o + 2] << 8) | (uint32_t)t[o + 3]);
  };
  const long ifd = u32(4);
  if (ifd < 8 || ifd + 2 > tl) return 1;
  const int cnt = u16(ifd);
  for (int e = 0; e < cnt; ++e) {
    const long o = ifd + 2 + 12l * e;
    if (o + 12 > tl) return 1;
    if (u16(o) == 0x0112) return u16(o + 8);
  }
  return 1;
}

// 0 ok, -1 corrupt, -2 unsupported (the caller decodes with PIL). The GPU pixel stage converts YCbCr;
// streams libjpeg (and so the reference's cv2.imdecode) takes as RGB -- an Adobe APP14 marker with
// transform 0, or no JFIF marker and component ids 'R', 'G', 'B' -- and streams with an EXIF rotation
// (cv2.imdecode applies it) are left to the fallback.
int parse(const uint8_t* d, long n, Jpeg& j) {
  if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return -1;
  long p = 2;
  bool sof = false;
  bool jfif = false;
  int adobe = -1;  // APP14 "Adobe" colour transform (-1: no such marker)
  while (p + 4 <= n) {
    if (d[p] != 0xFF) return -1;
    int m = d[p + 1];
    if (m == 0xFF) { ++p; continue; }  // fill byte
    p += 2;
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (m == 0xD9) return -1;  // EOI before the scan
    if (p + 2 > n) return -1;
    const int len = be16(d + p);
    if (len < 2 || p + len > n) return -1;
    const uint8_t* s = d + p + 2;
    const int sl = len - 2;
    switch (m) {
      case 0xDB: {  // DQT
        int q = 0;
        while (q < sl) {
          const int pq = s[q] >> 4, tq = s[q] & 15;
          if (tq > 3 || pq > 1) return -1;
          const int need = 1 + 64 * (pq + 1);
          if (q + need > sl) return -1;
          for (int i = 0; i < 64; ++i)
            j.qt[tq][kZigzag[i]] = pq ? (uint16_t)be16(s + q + 1 + 2 * i) : s[q + 1 + i];
          j.qt_present[tq] = true;
          q += need;
        }
        break;
      }
      case 0xC4: {  // DHT
        int q = 0;
        while (q < sl) {
          if (q + 17 > sl) return -1;
          const int tc = s[q] >> 4, th = s[q] & 15;
          if (tc > 1 || th > 3) return -1;
          Huff& hf = tc ? j.ac[th] : j.dc[th];
          int cnt = 0;
          hf.bits[0] = 0;
          for (int l = 1; l <= 16; ++l) {
            hf.bits[l] = s[q + l];
            cnt += hf.bits[l];
          }
          if (cnt > 256 || q + 17 + cnt > sl) return -1;
          std::memcpy(hf.vals, s + q + 17, cnt);
          if (!hf.build()) return -1;
          q += 17 + cnt;
        }
        break;
      }
      case 0xDD:  // DRI
        if (sl < 2) return -1;
        j.restart = be16(s);
        break;
      case 0xC0:
      case 0xC1: {  // baseline / extended sequential, Huffman
        if (sof || sl < 6) return -1;
        sof = true;
        if (s[0] != 8) return -2;
        j.height = be16(s + 1);
        j.width = be16(s + 3);
        j.ncomp = s[5];
        if (j.width <= 0 || j.height <= 0) return -2;  // DNL-defined height: unsupported
        // untrusted header: PIL's decompression-bomb bound (Image.MAX_IMAGE_PIXELS) before anything is
        // allocated from it -- the coefficient planes of a forged 65535 x 65535 header would be 25 GB
        if ((long)j.width * j.height > 89478485L) return -1;
        if (j.ncomp != 1 && j.ncomp != 3) return -2;
        if (sl < 6 + 3 * j.ncomp) return -1;
        for (int c = 0; c < j.ncomp; ++c) {
          Comp& cp = j.comp[c];
          cp.id = s[6 + 3 * c];
          cp.h = s[7 + 3 * c] >> 4;
          cp.v = s[7 + 3 * c] & 15;
          cp.tq = s[8 + 3 * c];
          if (cp.h < 1 || cp.h > 2 || cp.v < 1 || cp.v > 2 || cp.tq > 3) return -2;
        }
        break;
      }
      case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB: case 0xCD:
      case 0xCE: case 0xCF:
        return -2;  // progressive / lossless / hierarchical / arithmetic
      case 0xE0:  // APP0
        if (sl >= 5 && std::memcmp(s, "JFIF\0", 5) == 0) jfif = true;
        break;
      case 0xE1:  // APP1: EXIF orientation other than upright -> the fallback rotates like cv2.imdecode
        if (exif_orientation(s, sl) != 1) return -2;
        break;
      case 0xEE:  // APP14
        if (sl >= 12 && std::memcmp(s, "Adobe", 5) == 0) adobe = s[11];
        break;
      case 0xDA: {  // SOS
        if (!sof || sl < 1) return -1;
        if (j.ncomp == 3) {  // libjpeg's colour-space guess (jdapimin.c default_decompress_parms)
          const bool rgb = jfif ? false
                         : adobe >= 0 ? adobe == 0
                         : (j.comp[0].id == 'R' && j.comp[1].id == 'G' && j.comp[2].id == 'B');
          if (rgb) return -2;
        }
        const int ns = s[0];
        if (ns != j.ncomp || sl < 1 + 2 * ns + 3) return -2;  // one interleaved scan only
        for (int k = 0; k < ns; ++k) {
          const int id = s[1 + 2 * k];
          int c = 0;
          while (c < j.ncomp && j.comp[c].id != id) ++c;
          if (c == j.ncomp || c != k) return -2;
          j.comp[c].td = s[2 + 2 * k] >> 4;
          j.comp[c].ta = s[2 + 2 * k] & 15;
          if (j.comp[c].td > 3 || j.comp[c].ta > 3) return -1;
        }
        const int ss = s[1 + 2 * ns], se = s[2 + 2 * ns], ahl = s[3 + 2 * ns];
        if (ss != 0 || se != 63 || ahl != 0) return -2;
        j.scan_begin = p + len;
        // the scan ends at the first marker that is neither a stuffed 0xFF00 nor an RSTn. memchr jumps from
        // one 0xFF to the next (a byte loop over the ~100-300 KB of entropy data was ~40 us per pass on the
        // serving host, and the frame path parses every JPEG twice)
        long e = j.scan_begin;
        while (e + 1 < n) {
          const void* f = std::memchr(d + e, 0xFF, (size_t)(n - 1 - e));  // a hit leaves d[e + 1] readable
          if (!f) {
            e = n - 1;
            break;
          }
          e = (long)((const uint8_t*)f - d);
          const int mk = d[e + 1];
          if (mk == 0x00 || (mk >= 0xD0 && mk <= 0xD7)) { e += 2; continue; }
          if (mk == 0xFF) { ++e; continue; }
          break;
        }
        j.scan_end = std::min(e, n);
        // geometry
        j.hmax = j.vmax = 1;
        for (int c = 0; c < j.ncomp; ++c) {
          j.hmax = std::max(j.hmax, j.comp[c].h);
          j.vmax = std::max(j.vmax, j.comp[c].v);
        }
        if (j.ncomp == 1) {  // single component: blocks, not MCUs of the sampling factor
          j.comp[0].h = j.comp[0].v = j.hmax = j.vmax = 1;
        }
        // luma at full resolution (the GPU colour stage reads Y unscaled); chroma-only subsampling
        if (j.comp[0].h != j.hmax || j.comp[0].v != j.vmax) return -2;
        for (int c = 1; c < j.ncomp; ++c) {  // chroma 4:4:4, 4:2:2 (h2v1) or 4:2:0 (h2v2): the fancy upsamplers
          const int hr = j.hmax / j.comp[c].h, vr = j.vmax / j.comp[c].v;
          if (j.hmax % j.comp[c].h || j.vmax % j.comp[c].v || (vr == 2 && hr != 2)) return -2;
        }
        j.mcux = (j.width + 8 * j.hmax - 1) / (8 * j.hmax);
        j.mcuy = (j.height + 8 * j.vmax - 1) / (8 * j.vmax);
        long off = 0;
        for (int c = 0; c < j.ncomp; ++c) {
          Comp& cp = j.comp[c];
          if (!j.qt_present[cp.tq] || !j.dc[cp.td].present || !j.ac[cp.ta].present) return -1;
          cp.bw = j.mcux * cp.h;
          cp.bh = j.mcuy * cp.v;
          cp.plane_off = off;
          off += (long)cp.bw * cp.bh * 64;
        }
        j.total_coefs = off;
        return 0;
      }
      default:
        break;  // APPn, COM, DNL ... skipped
    }
    p += len;
  }
  return -1;
}

// ---- bit reader over one entropy-coded segment [p, end) (0xFF00 stuffing removed on the fly)
struct Bits {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t acc = 0;
  int n = 0;
  bool past_end = false;  // ran into a marker / the end: zeros are fed (as libjpeg does)
  void fill() {
    // fast path: 8 bytes without a 0xFF (no stuffing, no marker): take as many whole bytes as fit
    if (end - p >= 8) {
      uint64_t v;
      std::memcpy(&v, p, 8);
      v = __builtin_bswap64(v);
      const uint64_t x = ~v;
      if (((x - 0x0101010101010101ULL) & ~x & 0x8080808080808080ULL) == 0) {
        const int nb = (63 - n) >> 3;
        acc |= (v & (~0ULL << (64 - 8 * nb))) >> n;
        n += 8 * nb;
        p += nb;
        return;
      }
    }
    while (n <= 56) {
      uint32_t b = 0;
      if (p < end) {
        b = *p;
        if (b == 0xFF) {
          if (p + 1 < end && p[1] == 0x00) {
            p += 2;
          } else {  // a marker: stop here
            b = 0;
            past_end = true;
          }
        } else {
          ++p;
        }
      } else {
        past_end = true;
      }
      acc |= (uint64_t)b << (56 - n);
      n += 8;
    }
  }
  inline uint32_t peek(int k) {
    if (n < k) fill();
    return (uint32_t)(acc >> (64 - k));
  }
  inline void skip(int k) {
    acc <<= k;
    n -= k;
  }
  inline uint32_t get(int k) {
    if (k == 0) return 0;
    const uint32_t v = peek(k);
    skip(k);
    return v;
  }
};

inline int decode_huff(Bits& b, const Huff& h) {
  const uint32_t look = b.peek(9);
  const uint16_t e = h.look[look];
  if (e) {
    b.skip(e >> 8);
    return e & 0xFF;
  }
  // slow path: codes longer than 9 bits
  uint32_t code = b.peek(16);
  for (int l = 10; l <= 16; ++l) {
    const int c = (int)(code >> (16 - l));
    if (h.maxcode[l] >= 0 && c <= h.maxcode[l] && c >= h.mincode[l]) {
      b.skip(l);
      return h.vals[h.valptr[l] + c - h.mincode[l]];
    }
  }
  return -1;
}

inline int extend(uint32_t v, int s) { return (s && v < (1u << (s - 1))) ? (int)v - (1 << s) + 1 : (int)v; }

// decode MCUs [m0, m1) from one restart segment starting at `src`; 0 ok, -1 corrupt
int decode_segment(const Jpeg& j, const uint8_t* src, const uint8_t* end, long m0, long m1, int16_t* out) {
  Bits b{src, end};
  int pred[3] = {0, 0, 0};
  for (long m = m0; m < m1; ++m) {
    const int my = (int)(m / j.mcux), mx = (int)(m - (long)my * j.mcux);
    for (int c = 0; c < j.ncomp; ++c) {
      const Comp& cp = j.comp[c];
      const Huff& hd = j.dc[cp.td];
      const Huff& ha = j.ac[cp.ta];
      for (int by = 0; by < cp.v; ++by)
        for (int bx = 0; bx < cp.h; ++bx) {
          const long brow = (long)my * cp.v + by, bcol = (long)mx * cp.h + bx;
          int16_t* blk = out + cp.plane_off + (brow * cp.bw + bcol) * 64;
          std::memset(blk, 0, 64 * sizeof(int16_t));
          int s = decode_huff(b, hd);
          if (s < 0 || s > 11) return -1;
          pred[c] += extend(b.get(s), s);
          blk[0] = (int16_t)pred[c];
          for (int k = 1; k < 64;) {
            const int fa = ha.fast_ac[b.peek(9)];
            if (fa) {
              b.skip(fa & 15);
              k += (fa >> 4) & 15;
              if (k > 63) return -1;
              blk[kZigzag[k]] = (int16_t)(fa >> 8);
              ++k;
              continue;
            }
            const int rs = decode_huff(b, ha);
            if (rs < 0) return -1;
            const int r = rs >> 4;
            s = rs & 15;
            if (s == 0) {
              if (r != 15) break;  // EOB
              k += 16;
              continue;
            }
            k += r;
            if (k > 63) return -1;
            blk[kZigzag[k]] = (int16_t)extend(b.get(s), s);
            ++k;
          }
        }
    }
  }
  return 0;
}

}  // namespace

extern "C" {

// Header summary. info (int[24]): width, height, ncomp, hmax, vmax, mcux, mcuy, restart, segments,
// then per component (3 x 5): h, v, bw, bh, tq. Returns the coefficient count, or -1 corrupt / -2
// unsupported.
long rdp_jpeg_info(const uint8_t* d, long n, int* info) {
  Jpeg j;
  const int r = parse(d, n, j);
  if (r) return r;
  const long mcus = (long)j.mcux * j.mcuy;
  info[0] = j.width; info[1] = j.height; info[2] = j.ncomp; info[3] = j.hmax; info[4] = j.vmax;
  info[5] = j.mcux; info[6] = j.mcuy; info[7] = j.restart;
  info[8] = j.restart ? (int)((mcus + j.restart - 1) / j.restart) : 1;
  for (int c = 0; c < 3; ++c) {
    const Comp& cp = j.comp[c < j.ncomp ? c : 0];
    info[9 + 5 * c] = cp.h; info[10 + 5 * c] = cp.v; info[11 + 5 * c] = cp.bw; info[12 + 5 * c] = cp.bh;
    info[13 + 5 * c] = cp.tq;
  }
  return j.total_coefs;
}

// The pixel stage's geometry block (meta int32[32]: W, H, ncomp, hmax, vmax, total blocks; per component
// c at 8 + 8c: h, v, blocks per line, block rows, first block, plane byte offset, downsampled width,
// height) from rdp_jpeg_info's header summary `hi`.
void rdp_jpeg_meta(const int* hi, int* g) {
  const int W = hi[0], H = hi[1], nc = hi[2], hmax = hi[3], vmax = hi[4];
  for (int i = 0; i < 32; ++i) g[i] = 0;
  g[0] = W; g[1] = H; g[2] = nc; g[3] = hmax; g[4] = vmax;
  long blk = 0, pb = 0;
  for (int c = 0; c < nc; ++c) {
    const int h = hi[9 + 5 * c], v = hi[10 + 5 * c], bw = hi[11 + 5 * c], bh = hi[12 + 5 * c];
    int* q = g + 8 + 8 * c;
    q[0] = h; q[1] = v; q[2] = bw; q[3] = bh; q[4] = (int)blk; q[5] = (int)pb;
    q[6] = (W * h + hmax - 1) / hmax;
    q[7] = (H * v + vmax - 1) / vmax;
    blk += (long)bw * bh;
    pb += (long)bw * 8 * bh * 8;
  }
  g[5] = (int)blk;
}

// Entropy-decode into `coefs` (rdp_jpeg_info's count, int16, plane after plane, blocks row-major,
// natural order, quantized) and the component quantisation tables into qt[3][64] (natural order).
// Restart segments are decoded in parallel when `parallel`. 0 ok, -1 corrupt, -2 unsupported.
int rdp_jpeg_decode(const uint8_t* d, long n, int16_t* coefs, long ncoefs, uint16_t* qt, int parallel) {
  Jpeg j;
  int r = parse(d, n, j);
  if (r) return r;
  if (ncoefs < j.total_coefs) return -1;
  for (int c = 0; c < 3; ++c) std::memcpy(qt + 64 * c, j.qt[j.comp[c < j.ncomp ? c : 0].tq], 64 * sizeof(uint16_t));
  const long mcus = (long)j.mcux * j.mcuy;
  const uint8_t* beg = d + j.scan_begin;
  const uint8_t* end = d + j.scan_end;
  if (!j.restart) return decode_segment(j, beg, end, 0, mcus, coefs);
  // segment k starts after the k-th RSTn marker (RST markers are byte-aligned and never stuffed)
  const long nseg = (mcus + j.restart - 1) / j.restart;
  std::vector<const uint8_t*> starts(nseg + 1, end);
  starts[0] = beg;
  long k = 1;
  for (const uint8_t* p = beg; p + 1 < end && k < nseg;) {  // 0xFF to 0xFF (memchr), as in parse
    const uint8_t* f = (const uint8_t*)std::memchr(p, 0xFF, (size_t)(end - 1 - p));
    if (!f) break;
    if (f[1] >= 0xD0 && f[1] <= 0xD7) {
      starts[k++] = f + 2;
      p = f + 2;
    } else {
      p = f + 1;
    }
  }
  if (k != nseg) return -1;
  std::atomic<int> bad{0};
  auto seg = [&](int s) {
    const uint8_t* se = s + 1 < nseg ? starts[s + 1] - 2 : end;
    const long m0 = (long)s * j.restart, m1 = std::min(mcus, m0 + j.restart);
    if (decode_segment(j, starts[s], se, m0, m1, coefs) != 0) bad.store(1);
  };
  if (parallel) {
    rdp::host_pool().parallel_for((int)nseg, seg);
  } else {
    for (int s = 0; s < nseg; ++s) seg(s);
  }
  return bad.load() ? -1 : 0;
}

}  // extern "C"

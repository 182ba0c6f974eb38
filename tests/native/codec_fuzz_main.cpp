// Host sanitizer / fuzz driver for the native decoders of untrusted network input (SURVEY.md §5 "race
// detection / sanitizers"; the served request path of /root/reference/services/vision_analysis/server.py:
// 116-125 decodes client bytes with OpenCV): csrc/jpeg.cpp (baseline JPEG header + entropy decode),
// csrc/codecs.cpp (16-bit PNG header + banded inflate) and csrc/wire_parse.h (AnalysisRequest payloads).
// Built with -fsanitize=address,undefined (or thread) by tests/test_codec_sanitizers_cpu.py.
//
// usage: codec_fuzz <seed.jpg> <seed.png> <mutations> [threads]
//   1. the seeds decode (positive control);
//   2. <mutations> deterministic mutants of each seed (byte flips, truncation, inserted / duplicated
//      ranges, 0xFF marker bytes, bit noise) go through info + decode with output buffers sized exactly
//      from the header, so any write past the declared size is caught by the sanitizer;
//   3. AnalysisRequest messages built around the seeds, mutated the same way, go through the request
//      parser; returned payloads must lie inside the message;
//   4. [threads] > 1: that many threads decode the seeds concurrently (parallel restart segments / bands
//      on the shared host pool) -- the concurrency run for the thread sanitizer.
// Prints "<cases> cases, <failures> failures"; exit status 0 iff no failure.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../csrc/wire_parse.h"

extern "C" {
long rdp_jpeg_info(const uint8_t* d, long n, int* info);
int rdp_jpeg_decode(const uint8_t* d, long n, int16_t* coefs, long ncoefs, uint16_t* qt, int parallel);
int rdp_png_info(const uint8_t* d, long n, int* w, int* h, int* bd);
int rdp_png_decode(const uint8_t* d, long n, uint8_t* out, long out_bytes, int parallel);
}

namespace {

std::vector<uint8_t> read_file(const char* path) {
  std::vector<uint8_t> v;
  FILE* f = std::fopen(path, "rb");
  if (!f) return v;
  uint8_t buf[65536];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) v.insert(v.end(), buf, buf + n);
  std::fclose(f);
  return v;
}

struct Rng {  // xorshift64*: deterministic mutants
  uint64_t s;
  uint64_t next() {
    s ^= s >> 12; s ^= s << 25; s ^= s >> 27;
    return s * 2685821657736338717ull;
  }
  size_t below(size_t n) { return n ? (size_t)(next() % n) : 0; }
};

std::vector<uint8_t> mutate(const std::vector<uint8_t>& in, Rng& r) {
  std::vector<uint8_t> v = in;
  const int k = 1 + (int)r.below(6);
  for (int i = 0; i < k && !v.empty(); ++i) {
    const size_t at = r.below(v.size());
    switch (r.below(7)) {
      case 0: v[at] = (uint8_t)r.next(); break;                       // random byte
      case 1: v[at] ^= (uint8_t)(1u << r.below(8)); break;            // bit flip
      case 2: v.resize(at); break;                                    // truncation
      case 3: v.insert(v.begin() + at, 0xFF); break;                  // a marker prefix
      case 4: {                                                       // duplicated range
        const size_t len = std::min<size_t>(1 + r.below(64), v.size() - at);
        std::vector<uint8_t> seg(v.begin() + at, v.begin() + at + len);
        v.insert(v.begin() + r.below(v.size()), seg.begin(), seg.end());
        break;
      }
      case 5: v.erase(v.begin() + at, v.begin() + std::min(v.size(), at + 1 + r.below(16))); break;
      default: {  // a header-sized field set to an extreme (lengths, dimensions)
        const uint8_t x[4] = {0x00, 0xFF, 0x7F, 0x80};
        v[at] = x[r.below(4)];
        if (at + 1 < v.size()) v[at + 1] = x[r.below(4)];
      }
    }
  }
  return v;
}

long g_cases = 0, g_fail = 0;

void fail(const char* what, long i) {
  ++g_fail;
  std::printf("FAIL %s (case %ld)\n", what, i);
}

// header + decode with an output buffer of exactly the declared size; returns the decode status
int try_jpeg(const std::vector<uint8_t>& v, int parallel) {
  int info[24];
  const long nco = rdp_jpeg_info(v.data(), (long)v.size(), info);
  if (nco <= 0 || nco > (64L << 20)) return -100;
  std::vector<int16_t> coefs((size_t)nco);
  uint16_t qt[3 * 64];
  return rdp_jpeg_decode(v.data(), (long)v.size(), coefs.data(), nco, qt, parallel);
}

int try_png(const std::vector<uint8_t>& v, int parallel) {
  int w = 0, h = 0, bd = 0;
  if (rdp_png_info(v.data(), (long)v.size(), &w, &h, &bd) != 0) return -100;
  if (w <= 0 || h <= 0 || (bd != 8 && bd != 16) || (long)w * h > (16L << 20)) return -101;
  const long bytes = (long)w * h * (bd / 8);
  std::vector<uint8_t> out((size_t)bytes);
  return rdp_png_decode(v.data(), (long)v.size(), out.data(), bytes, parallel);
}

void put_varint(std::vector<uint8_t>& o, uint64_t v) {
  while (v >= 0x80) { o.push_back((uint8_t)(v | 0x80)); v >>= 7; }
  o.push_back((uint8_t)v);
}

std::vector<uint8_t> image_msg(const std::vector<uint8_t>& data, int w, int h) {
  std::vector<uint8_t> o;
  o.push_back(0x0A); put_varint(o, data.size()); o.insert(o.end(), data.begin(), data.end());
  o.push_back(0x10); put_varint(o, (uint64_t)w);
  o.push_back(0x18); put_varint(o, (uint64_t)h);
  return o;
}

std::vector<uint8_t> request_msg(const std::vector<uint8_t>& jpg, const std::vector<uint8_t>& png) {
  std::vector<uint8_t> o;
  const auto c = image_msg(jpg, 640, 480), d = image_msg(png, 640, 480);
  o.push_back(0x0A); put_varint(o, c.size()); o.insert(o.end(), c.begin(), c.end());
  o.push_back(0x12); put_varint(o, d.size()); o.insert(o.end(), d.begin(), d.end());
  return o;
}

bool inside(const uint8_t* p, size_t n, const std::vector<uint8_t>& buf) {
  const uint8_t* b = buf.data();
  return p >= b && n <= buf.size() && (size_t)(p - b) <= buf.size() - n;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::printf("usage: codec_fuzz <seed.jpg> <seed.png> <mutations> [threads]\n");
    return 2;
  }
  const std::vector<uint8_t> jpg = read_file(argv[1]), png = read_file(argv[2]);
  const long muts = std::atol(argv[3]);
  const int threads = argc > 4 ? std::atoi(argv[4]) : 1;
  if (jpg.empty() || png.empty()) {
    std::printf("cannot read the seeds\n");
    return 2;
  }
  // 1. positive controls
  ++g_cases;
  if (try_jpeg(jpg, 1) != 0) fail("seed JPEG does not decode", 0);
  ++g_cases;
  if (try_png(png, 1) != 0) fail("seed PNG does not decode", 0);
  const std::vector<uint8_t> req = request_msg(jpg, png);
  {
    ++g_cases;
    const uint8_t *c, *d;
    size_t cn, dn;
    if (!rdp_wire::parse_request(req.data(), req.size(), c, cn, d, dn) || cn != jpg.size() || dn != png.size() ||
        std::memcmp(c, jpg.data(), cn) != 0 || std::memcmp(d, png.data(), dn) != 0)
      fail("seed request does not parse to its payloads", 0);
  }
  // 2. mutated codec inputs (statuses are free; memory errors are the sanitizer's to report)
  Rng r{0x9E3779B97F4A7C15ull};
  long jpeg_ok = 0, png_ok = 0;
  for (long i = 0; i < muts; ++i) {
    const auto mj = mutate(jpg, r);
    ++g_cases;
    jpeg_ok += try_jpeg(mj, (int)(i & 1)) == 0;
    const auto mp = mutate(png, r);
    ++g_cases;
    png_ok += try_png(mp, (int)(i & 1)) == 0;
  }
  // 3. mutated requests: a parse either declines or returns payloads inside the message
  for (long i = 0; i < muts; ++i) {
    const auto m = mutate(req, r);
    ++g_cases;
    const uint8_t *c, *d;
    size_t cn, dn;
    if (rdp_wire::parse_request(m.data(), m.size(), c, cn, d, dn) && (!inside(c, cn, m) || !inside(d, dn, m)))
      fail("parsed payload outside the message", i);
  }
  // 4. concurrent decodes on the shared host pool
  if (threads > 1) {
    std::vector<std::thread> ts;
    std::vector<int> bad(threads, 0);
    for (int t = 0; t < threads; ++t)
      ts.emplace_back([&, t] {
        for (int i = 0; i < 40; ++i) {
          if (try_jpeg(jpg, 1) != 0) bad[t] = 1;
          if (try_png(png, 1) != 0) bad[t] = 1;
        }
      });
    for (auto& t : ts) t.join();
    for (int t = 0; t < threads; ++t) {
      ++g_cases;
      if (bad[t]) fail("concurrent decode of a seed failed", t);
    }
  }
  std::printf("%ld cases, %ld failures (mutants decoded: %ld JPEG, %ld PNG)\n", g_cases, g_fail, jpeg_ok, png_ok);
  return g_fail ? 1 : 0;
}

// evofab.vision.AnalysisRequest wire bytes -> its two Image.data payloads, read in place.
//
// /root/reference/protos/vision.proto:14-24: Image{bytes data = 1; int32 width = 2; int32 height = 3},
// AnalysisRequest{Image color_image = 1; Image depth_image = 2}. The native serving path
// (serve_runtime.cpp FrameRunner / BatchRunner submit_request) parses requests here without protobuf,
// without copies and without the interpreter lock. The bytes come from the network: every read is
// bounded by the end pointer, and a message this parser does not take (a malformed one, or one without
// both payloads) returns false -- the caller then parses it with protobuf in Python. Header-only so the
// host sanitizer / fuzz build (tests/native/codec_fuzz_main.cpp) compiles it without HIP.
#pragma once

#include <cstddef>
#include <cstdint>

namespace rdp_wire {

inline bool read_varint(const uint8_t*& p, const uint8_t* e, uint64_t& v) {
  v = 0;
  for (int sh = 0; sh < 64 && p < e; sh += 7) {
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7f) << sh;
    if (!(b & 0x80)) return true;
  }
  return false;
}

inline bool skip_field(const uint8_t*& p, const uint8_t* e, int wt) {
  uint64_t v;
  switch (wt) {
    case 0: return read_varint(p, e, v);
    case 1: if (e - p < 8) return false; p += 8; return true;
    case 2: if (!read_varint(p, e, v) || (uint64_t)(e - p) < v) return false; p += v; return true;
    case 5: if (e - p < 4) return false; p += 4; return true;
    default: return false;
  }
}

// Image message in [p, e): its data field (proto3: the last occurrence wins)
inline bool image_data(const uint8_t* p, const uint8_t* e, const uint8_t*& d, size_t& n) {
  d = nullptr;
  n = 0;
  while (p < e) {
    uint64_t key;
    if (!read_varint(p, e, key)) return false;
    const int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f == 1 && wt == 2) {
      uint64_t len;
      if (!read_varint(p, e, len) || (uint64_t)(e - p) < len) return false;
      d = p;
      n = (size_t)len;
      p += len;
    } else if (!skip_field(p, e, wt)) {
      return false;
    }
  }
  return true;
}

// true with both payloads (non-empty) found; false: not a message this parser takes
inline bool parse_request(const uint8_t* p, size_t size, const uint8_t*& c, size_t& cn, const uint8_t*& d,
                          size_t& dn) {
  const uint8_t* e = p + size;
  c = d = nullptr;
  cn = dn = 0;
  while (p < e) {
    uint64_t key;
    if (!read_varint(p, e, key)) return false;
    const int f = (int)(key >> 3), wt = (int)(key & 7);
    if ((f == 1 || f == 2) && wt == 2) {
      uint64_t len;
      if (!read_varint(p, e, len) || (uint64_t)(e - p) < len) return false;
      if (!image_data(p, p + len, f == 1 ? c : d, f == 1 ? cn : dn)) return false;
      p += len;
    } else if (!skip_field(p, e, wt)) {
      return false;
    }
  }
  return c != nullptr && d != nullptr && cn > 0 && dn > 0;
}

}  // namespace rdp_wire

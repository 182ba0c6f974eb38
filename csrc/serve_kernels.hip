// Serving-path pre/post-processing kernels (per frame, graph-capturable).
//
// preprocess: replaces torchvision ToTensor() + Resize((256,256), antialias=True) + BGR->RGB (or RGB
//   input as decoded by the server, rgb = 1) of
//   /root/reference/services/vision_analysis/server.py:107-110,120-121: u8 BGR HWC -> /255 ->
//   antialiased bilinear (triangle filter, support = scale, normalized weights, torch
//   _upsample_bilinear2d_aa semantics; weight tables precomputed on the host) -> bf16 NHWC with
//   8 channels (3 RGB + 5 zero) = the packed first-layer input of the native U-Net.
// mask_upsample: replaces (sigmoid(logits) > 0.5) -> cv2.resize(INTER_NEAREST) -> count_nonzero
//   (server.py:124-125,133): u8 {0,1} mask at the camera resolution + coverage count (atomics).
#include "common.h"
#include <algorithm>
#include <stdlib.h>

#define AA_MAXTAP 16

struct AATable {  // per output index: first input index, number of taps, weights
  int start[256];
  int size[256];
  float w[256][AA_MAXTAP];
};

RDP_DEV void preprocess_body(const uint8_t* __restrict__ bgr, int H, int W, const int* __restrict__ ystart,
                             const int* __restrict__ ysize, const float* __restrict__ yw,
                             const int* __restrict__ xstart, const int* __restrict__ xsize,
                             const float* __restrict__ xw, int OH, int OW, int rgb, u16* __restrict__ out) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= OH * OW) return;
  const int oy = o / OW, ox = o - oy * OW;
  const int y0 = ystart[oy], ny = ysize[oy], x0 = xstart[ox], nx = xsize[ox];
  float r = 0.f, g = 0.f, b = 0.f;
  for (int j = 0; j < ny; ++j) {
    const float wy = yw[oy * AA_MAXTAP + j];
    const uint8_t* row = bgr + ((size_t)(y0 + j) * W + x0) * 3;
    float rr = 0.f, gg = 0.f, bb = 0.f;
    for (int i = 0; i < nx; ++i) {
      const float wx = xw[ox * AA_MAXTAP + i];
      bb += wx * (float)row[i * 3 + 0];
      gg += wx * (float)row[i * 3 + 1];
      rr += wx * (float)row[i * 3 + 2];
    }
    r += wy * rr;
    g += wy * gg;
    b += wy * bb;
  }
  if (rgb) {  // input already RGB (the server decodes JPEG straight to RGB): channels 0 / 2 swap roles
    const float t = r;
    r = b;
    b = t;
  }
  const float inv = 1.0f / 255.0f;
  uint4 v;
  v.x = pack2bf(r * inv, g * inv);
  v.y = pack2bf(b * inv, 0.f);
  v.z = 0u;
  v.w = 0u;
  *(uint4*)(out + (size_t)o * 8) = v;
}

__global__ void preprocess_kernel(const uint8_t* __restrict__ bgr, int H, int W, const int* __restrict__ ystart,
                                  const int* __restrict__ ysize, const float* __restrict__ yw,
                                  const int* __restrict__ xstart, const int* __restrict__ xsize,
                                  const float* __restrict__ xw, int OH, int OW, int rgb, u16* __restrict__ out) {
  preprocess_body(bgr, H, W, ystart, ysize, yw, xstart, xsize, xw, OH, OW, rgb, out);
}

// up to 4 frames of a serving batch in one launch (blockIdx.y = frame; serve/engine.py BatchEngine)
struct PreFrames {
  const uint8_t* bgr[4];
  u16* out[4];
};
__global__ void preprocess_batch_kernel(const PreFrames f, int H, int W, const int* __restrict__ ystart,
                                        const int* __restrict__ ysize, const float* __restrict__ yw,
                                        const int* __restrict__ xstart, const int* __restrict__ xsize,
                                        const float* __restrict__ xw, int OH, int OW, int rgb) {
  preprocess_body(f.bgr[blockIdx.y], H, W, ystart, ysize, yw, xstart, xsize, xw, OH, OW, rgb, f.out[blockIdx.y]);
}

// nearest upsample of the model-resolution mask to (H, W) + coverage count.
// src index = min(floor(dst * (in/out)), in-1) in double, like cv::resize INTER_NEAREST.
__global__ void mask_upsample_kernel(const uint8_t* __restrict__ m, int mh, int mw, uint8_t* __restrict__ out,
                                     int H, int W, double sy, double sx, unsigned* __restrict__ count) {
  __shared__ unsigned wc[4];
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned v = 0;
  if (p < H * W) {
    const int y = p / W, x = p - y * W;
    int iy = (int)floor((double)y * sy), ix = (int)floor((double)x * sx);
    iy = min(iy, mh - 1);
    ix = min(ix, mw - 1);
    v = m[iy * mw + ix];
    out[p] = (uint8_t)v;
  }
  // block count -> one atomic per block
  unsigned long long b = __ballot(v != 0);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = (unsigned)__popcll(b);
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(count, wc[0] + wc[1] + wc[2] + wc[3]);
}

__global__ void zero_u32_kernel(unsigned* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0;
}

extern "C" {
int rdp_preprocess(const void* bgr, int H, int W, const int* ystart, const int* ysize, const float* yw,
                   const int* xstart, const int* xsize, const float* xw, int OH, int OW, int rgb, void* out,
                   hipStream_t s) {
  const int n = OH * OW;
  hipLaunchKernelGGL(preprocess_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const uint8_t*)bgr, H, W, ystart,
                     ysize, yw, xstart, xsize, xw, OH, OW, rgb, (u16*)out);
  return 0;
}

int rdp_preprocess_batch(int n, const void* const* bgr, int H, int W, const int* ystart, const int* ysize,
                         const float* yw, const int* xstart, const int* xsize, const float* xw, int OH, int OW, int rgb,
                         void* const* out, hipStream_t s) {
  if (n < 1 || n > 4) return -1;
  PreFrames f;
  for (int i = 0; i < 4; ++i) {
    f.bgr[i] = (const uint8_t*)bgr[i < n ? i : 0];
    f.out[i] = (u16*)out[i < n ? i : 0];
  }
  const int np = OH * OW;
  hipLaunchKernelGGL(preprocess_batch_kernel, dim3((np + 255) / 256, n), dim3(256), 0, s, f, H, W, ystart, ysize, yw,
                     xstart, xsize, xw, OH, OW, rgb);
  return 0;
}

int rdp_mask_upsample(const void* m, int mh, int mw, void* out, int H, int W, unsigned* count, hipStream_t s) {
  hipLaunchKernelGGL(zero_u32_kernel, dim3(1), dim3(64), 0, s, count, 1);
  const double sy = 1.0 / ((double)H / (double)mh), sx = 1.0 / ((double)W / (double)mw);
  hipLaunchKernelGGL(mask_upsample_kernel, dim3((H * W + 255) / 256), dim3(256), 0, s, (const uint8_t*)m, mh, mw,
                     (uint8_t*)out, H, W, sy, sx, count);
  return 0;
}
}

// ---------------------------------------------------------------------------------------------
// JPEG pixel stage on the GPU (the entropy decode is csrc/jpeg.cpp on the host). Follows libjpeg's
// default decode of the reference server's cv2.imdecode (server.py:117): dequantisation + the ISLOW
// integer IDCT (13-bit constants, 2 extra bits in pass 1, +128 and clamp), "fancy" (triangle) chroma
// upsampling for 2x2 / 2x1 subsampling with edge replication, and the fixed-point YCbCr -> RGB of
// jdcolor.c (16-bit scale). geo: see bindings.cpp jpeg_decode.
#define JF_0_298631336 2446
#define JF_0_390180644 3196
#define JF_0_541196100 4433
#define JF_0_765366865 6270
#define JF_0_899976223 7373
#define JF_1_175875602 9633
#define JF_1_501321110 12299
#define JF_1_847759065 15137
#define JF_1_961570560 16069
#define JF_2_053119869 16819
#define JF_2_562915447 20995
#define JF_3_072711026 25172

// one 1-D ISLOW pass over v[0..7] (stride 1); results before the final descale: out[i] = value << shift
RDP_DEV void jidct_1d(const int* v, int& e0, int& e1, int& e2, int& e3, int& o0, int& o1, int& o2, int& o3) {
  int z2 = v[2], z3 = v[6];
  int z1 = (z2 + z3) * JF_0_541196100;
  const int t2 = z1 + z3 * (-JF_1_847759065);
  const int t3 = z1 + z2 * JF_0_765366865;
  z2 = v[0];
  z3 = v[4];
  const int t0 = (z2 + z3) << 13;
  const int t1 = (z2 - z3) << 13;
  e0 = t0 + t3;  // tmp10
  e3 = t0 - t3;  // tmp13
  e1 = t1 + t2;  // tmp11
  e2 = t1 - t2;  // tmp12
  int a0 = v[7], a1 = v[5], a2 = v[3], a3 = v[1];
  z1 = a0 + a3;
  z2 = a1 + a2;
  z3 = a0 + a2;
  int z4 = a1 + a3;
  const int z5 = (z3 + z4) * JF_1_175875602;
  a0 *= JF_0_298631336;
  a1 *= JF_2_053119869;
  a2 *= JF_3_072711026;
  a3 *= JF_1_501321110;
  z1 *= -JF_0_899976223;
  z2 *= -JF_2_562915447;
  z3 *= -JF_1_961570560;
  z4 *= -JF_0_390180644;
  z3 += z5;
  z4 += z5;
  o0 = a0 + z1 + z3;  // tmp0
  o1 = a1 + z2 + z4;  // tmp1
  o2 = a2 + z2 + z3;  // tmp2
  o3 = a3 + z1 + z4;  // tmp3
}

RDP_DEV void jpeg_idct_body(const int16_t* __restrict__ coefs, const int* __restrict__ geo,
                            const int* __restrict__ qt, uint8_t* __restrict__ planes) {
  __shared__ int ws[32][64];
  const int lb = threadIdx.x >> 3, k = threadIdx.x & 7;
  const int jb = blockIdx.x * 32 + lb;
  const int nc = geo[2];
  const bool act = jb < geo[5];
  int c = 0;
  if (nc > 1 && jb >= geo[8 + 8 + 4]) c = 1;
  if (nc > 2 && jb >= geo[8 + 16 + 4]) c = 2;
  const int* g = geo + 8 + 8 * c;
  if (act) {  // pass 1: column k, dequantised, results scaled by 2^2 (PASS1_BITS)
    const int16_t* in = coefs + (long)jb * 64;
    const int* q = qt + 64 * c;
    int v[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = (int)in[r * 8 + k] * q[r * 8 + k];
    int e0, e1, e2, e3, o0, o1, o2, o3;
    jidct_1d(v, e0, e1, e2, e3, o0, o1, o2, o3);
    constexpr int S = 13 - 2, R = 1 << (S - 1);
    ws[lb][0 * 8 + k] = (e0 + o3 + R) >> S;
    ws[lb][7 * 8 + k] = (e0 - o3 + R) >> S;
    ws[lb][1 * 8 + k] = (e1 + o2 + R) >> S;
    ws[lb][6 * 8 + k] = (e1 - o2 + R) >> S;
    ws[lb][2 * 8 + k] = (e2 + o1 + R) >> S;
    ws[lb][5 * 8 + k] = (e2 - o1 + R) >> S;
    ws[lb][3 * 8 + k] = (e3 + o0 + R) >> S;
    ws[lb][4 * 8 + k] = (e3 - o0 + R) >> S;
  }
  __syncthreads();
  if (!act) return;
  int v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = ws[lb][k * 8 + i];
  int e0, e1, e2, e3, o0, o1, o2, o3;
  jidct_1d(v, e0, e1, e2, e3, o0, o1, o2, o3);
  constexpr int S = 13 + 2 + 3, R = 1 << (S - 1);
  auto px = [](int x) -> uint32_t { return (uint32_t)min(max(((x + R) >> S) + 128, 0), 255); };
  const uint32_t p0 = px(e0 + o3), p7 = px(e0 - o3), p1 = px(e1 + o2), p6 = px(e1 - o2);
  const uint32_t p2 = px(e2 + o1), p5 = px(e2 - o1), p3 = px(e3 + o0), p4 = px(e3 - o0);
  const int lbi = jb - g[4], bw = g[2];
  const int by = lbi / bw, bx = lbi - by * bw;
  uint8_t* dst = planes + g[5] + (long)(by * 8 + k) * (bw * 8) + bx * 8;
  *(uint2*)dst = make_uint2(p0 | p1 << 8 | p2 << 16 | p3 << 24, p4 | p5 << 8 | p6 << 16 | p7 << 24);
}

RDP_DEV int jpeg_chroma(const uint8_t* __restrict__ planes, const int* g, int hmax, int vmax, int y, int x) {
  const uint8_t* base = planes + g[5];
  const int stride = g[2] * 8, dsw = g[6], dsh = g[7];
  const int hr = hmax / g[0], vr = vmax / g[1];
  if (hr == 1 && vr == 1) return base[y * stride + x];
  if (hr == 2 && vr == 1) {  // h2v1 fancy
    const int cx = x >> 1;
    const int v0 = base[y * stride + cx];
    if ((x & 1) == 0) return (3 * v0 + base[y * stride + max(cx - 1, 0)] + 1) >> 2;
    return (3 * v0 + base[y * stride + min(cx + 1, dsw - 1)] + 2) >> 2;
  }
  if (hr == 2 && vr == 2) {  // h2v2 fancy: vertical 3:1 column sums, then horizontal 3:1
    const int cy = y >> 1, ny = (y & 1) ? min(cy + 1, dsh - 1) : max(cy - 1, 0);
    const int cx = x >> 1;
    auto colsum = [&](int cc) { return 3 * base[cy * stride + cc] + base[ny * stride + cc]; };
    const int t = colsum(cx);
    if ((x & 1) == 0) return (3 * t + colsum(max(cx - 1, 0)) + 8) >> 4;
    return (3 * t + colsum(min(cx + 1, dsw - 1)) + 7) >> 4;
  }
  return base[(y / vr) * stride + x / hr];
}

RDP_DEV void jpeg_color_body(const uint8_t* __restrict__ planes, const int* __restrict__ geo, int H, int W,
                             uint8_t* __restrict__ rgb) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= H * W) return;
  const int y = p / W, x = p - y * W;
  const int* g0 = geo + 8;
  const int yy = planes[g0[5] + (long)y * (g0[2] * 8) + x];
  int r = yy, gg = yy, b = yy;
  if (geo[2] == 3) {
    const int cb = jpeg_chroma(planes, geo + 16, geo[3], geo[4], y, x) - 128;
    const int cr = jpeg_chroma(planes, geo + 24, geo[3], geo[4], y, x) - 128;
    r = yy + ((91881 * cr + 32768) >> 16);
    gg = yy + ((-22554 * cb + 32768 - 46802 * cr) >> 16);
    b = yy + ((116130 * cb + 32768) >> 16);
  }
  uint8_t* o = rgb + (long)p * 3;
  o[0] = (uint8_t)min(max(r, 0), 255);
  o[1] = (uint8_t)min(max(gg, 0), 255);
  o[2] = (uint8_t)min(max(b, 0), 255);
}

__global__ __launch_bounds__(256) void jpeg_idct_kernel(const int16_t* __restrict__ coefs, const int* __restrict__ geo,
                                                        const int* __restrict__ qt, uint8_t* __restrict__ planes) {
  jpeg_idct_body(coefs, geo, qt, planes);
}
__global__ __launch_bounds__(256) void jpeg_color_kernel(const uint8_t* __restrict__ planes, const int* __restrict__ geo,
                                                         int H, int W, uint8_t* __restrict__ rgb) {
  jpeg_color_body(planes, geo, H, W, rgb);
}
struct JpegFrames {
  const int16_t* coefs[4];
  const int* geo[4];
  const int* qt[4];
  uint8_t* planes[4];
  uint8_t* rgb[4];
};
__global__ __launch_bounds__(256) void jpeg_idct_batch_kernel(const JpegFrames f) {
  const int i = blockIdx.y;
  jpeg_idct_body(f.coefs[i], f.geo[i], f.qt[i], f.planes[i]);
}
__global__ __launch_bounds__(256) void jpeg_color_batch_kernel(const JpegFrames f, int H, int W) {
  const int i = blockIdx.y;
  jpeg_color_body(f.planes[i], f.geo[i], H, W, f.rgb[i]);
}

extern "C" {
// the JPEG pixel stage of n <= 4 frames (each its coefficient / meta / planes / RGB buffers) in 2 launches
int rdp_jpeg_gpu_batch(int n, const void* const* coefs, const int* const* geo, const int* const* qt,
                       void* const* planes, int H, int W, int max_blocks, void* const* rgb, hipStream_t s) {
  if (n < 1 || n > 4) return -1;
  JpegFrames f;
  for (int i = 0; i < 4; ++i) {
    const int j = i < n ? i : 0;
    f.coefs[i] = (const int16_t*)coefs[j];
    f.geo[i] = geo[j];
    f.qt[i] = qt[j];
    f.planes[i] = (uint8_t*)planes[j];
    f.rgb[i] = (uint8_t*)rgb[j];
  }
  hipLaunchKernelGGL(jpeg_idct_batch_kernel, dim3((max_blocks + 31) / 32, n), dim3(256), 0, s, f);
  hipLaunchKernelGGL(jpeg_color_batch_kernel, dim3((H * W + 255) / 256, n), dim3(256), 0, s, f, H, W);
  return 0;
}

// coefficient / plane capacity for frames of H x W (any supported sampling: Y and chroma planes at most
// MCU-padded to 16 x 16)
long rdp_jpeg_max_coefs(int H, int W) { return 3L * ((W + 15) / 16 * 16) * ((H + 15) / 16 * 16); }
long rdp_jpeg_plane_bytes(int H, int W) { return rdp_jpeg_max_coefs(H, W); }

int rdp_jpeg_gpu(const void* coefs, const int* geo, const int* qt, void* planes, int H, int W, int max_blocks, void* rgb,
                 hipStream_t s) {
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3((max_blocks + 31) / 32), dim3(256), 0, s, (const int16_t*)coefs, geo, qt,
                     (uint8_t*)planes);
  hipLaunchKernelGGL(jpeg_color_kernel, dim3((H * W + 255) / 256), dim3(256), 0, s, (const uint8_t*)planes, geo, H, W,
                     (uint8_t*)rgb);
  return 0;
}
}

// Frame upload as a kernel on the frame's own queue: pinned host staging -> device, every 16-B chunk
// one lane (a 640x480x3 colour frame is 57,600 chunks = 225 blocks, all in flight at once). Measured
// against the DMA-engine copy it replaces (profiles/serve_experiments.md): the engine copy took 31 us
// for 921 KB and the preprocess kernel started ~10 us after it ended (the copy engine's completion
// signal -> compute queue hand-off), 40 us of every frame before its first kernel.
__global__ __launch_bounds__(256) void h2d_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                       long n16, const uint8_t* __restrict__ tsrc,
                                                       uint8_t* __restrict__ tdst, int ntail) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) dst[i] = src[i];
  if (i < ntail) tdst[i] = tsrc[i];
}

// U chunks per lane, strided by the grid (each load instruction of a wave still covers 1 KiB contiguous)
__global__ __launch_bounds__(256) void h2d_copy4_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                        long n16, const uint8_t* __restrict__ tsrc,
                                                        uint8_t* __restrict__ tdst, int ntail) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x, str = (long)gridDim.x * 256;
  uint4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (i + u * str < n16) v[u] = src[i + u * str];
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (i + u * str < n16) dst[i + u * str] = v[u];
  if (i < ntail) tdst[i] = tsrc[i];
}

extern "C" int rdp_h2d_copy(const void* src, void* dst, long bytes, hipStream_t s) {
  if (bytes <= 0) return 0;
  if (((uintptr_t)src | (uintptr_t)dst) & 15) return -1;
  const long n16 = bytes / 16;
  const int ntail = (int)(bytes - n16 * 16);
  // 4 chunks per lane by default (engine GPU p50 0.385 vs 0.387 ms in two interleaved rounds,
  // profiles/serve_experiments.md); RDP_H2D_VEC=1: one chunk per lane
  static const int vec = [] {
    const char* e = getenv("RDP_H2D_VEC");
    return e && atoi(e) == 1 ? 1 : 4;
  }();
  const long lanes = vec == 4 ? std::max<long>((n16 + 3) / 4, ntail) : std::max<long>(n16, ntail);
  const long blocks = std::max<long>(1, (lanes + 255) / 256);
  if (vec == 4)
    hipLaunchKernelGGL(h2d_copy4_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint4*)src, (uint4*)dst, n16,
                       (const uint8_t*)src + n16 * 16, (uint8_t*)dst + n16 * 16, ntail);
  else
    hipLaunchKernelGGL(h2d_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint4*)src, (uint4*)dst, n16,
                       (const uint8_t*)src + n16 * 16, (uint8_t*)dst + n16 * 16, ntail);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Several host -> device uploads in ONE launch (the batched serving path: every frame of a batch has its
// colour / JPEG coefficients, metadata and depth staged in pinned memory): blockIdx.y = segment, each
// lane moves 4 16-byte chunks strided by the segment's grid row, plus the segment's byte tail.
struct CopySegs {
  const uint8_t* src[16];
  uint8_t* dst[16];
  long bytes[16];
};

__global__ __launch_bounds__(256) void h2d_copy_multi_kernel(CopySegs g) {
  const int sg = blockIdx.y;
  const long bytes = g.bytes[sg];
  const long n16 = bytes / 16;
  const uint4* __restrict__ src = (const uint4*)g.src[sg];
  uint4* __restrict__ dst = (uint4*)g.dst[sg];
  const long i = (long)blockIdx.x * 256 + threadIdx.x, str = (long)gridDim.x * 256;
  for (long b = i; b < n16; b += 4 * str) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (b + u * str < n16) v[u] = src[b + u * str];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (b + u * str < n16) dst[b + u * str] = v[u];
  }
  const long t = n16 * 16 + i;
  if (i < 16 && t < bytes) g.dst[sg][t] = g.src[sg][t];
}

// n <= 16 segments, every src / dst 16-byte aligned (returns -1, nothing launched, otherwise)
extern "C" int rdp_h2d_copy_multi(const void* const* src, void* const* dst, const long* bytes, int n, hipStream_t s) {
  if (n <= 0) return 0;
  if (n > 16) return -1;
  CopySegs g;
  long most = 0;
  for (int k = 0; k < n; ++k) {
    if ((((uintptr_t)src[k] | (uintptr_t)dst[k]) & 15) || bytes[k] < 0) return -1;
    g.src[k] = (const uint8_t*)src[k];
    g.dst[k] = (uint8_t*)dst[k];
    g.bytes[k] = bytes[k];
    most = std::max(most, bytes[k]);
  }
  const long lanes = std::max<long>((most / 16 + 3) / 4, 16);
  const long bx = std::max<long>(1, (lanes + 255) / 256);
  hipLaunchKernelGGL(h2d_copy_multi_kernel, dim3((unsigned)bx, (unsigned)n), dim3(256), 0, s, g);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

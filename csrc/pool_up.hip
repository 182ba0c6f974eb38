// MaxPool2d(2) and bilinear x2 upsampling (align_corners=True) with zero-pad placement, NHWC bf16.
//
// Reference ops: nn.MaxPool2d(2) in Down (/root/reference/pkg/segmentation_model.py:47) and
// nn.Upsample(scale_factor=2, mode='bilinear', align_corners=True) + F.pad in Up.forward (:61,68-74).
// Semantics preserved:
//   * maxpool: floor mode; backward routes the gradient to the FIRST maximum of each 2x2 window in
//     row-major order (NaN wins), as torch does; the skip-connection gradient is added in the same
//     pass (d a = pool_bwd(d p) + d skip), so the encoder activation's gradient is written once.
//   * upsample: src = dst * (in-1)/(out-1) in fp32 (torch area_pixel_compute_source_index),
//     i1 = i0 + (i0 < in-1); the x2 output is placed at offset (oy, ox) inside the skip's H2 x W2
//     (F.pad with [dx//2, dx-dx//2, dy//2, dy-dy//2]); the rest is zero. Backward is a
//     deterministic gather (no atomics) that re-derives the forward's exact index/weight arithmetic.
#include "common.h"
#include <algorithm>

RDP_DEV void unpack8f(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = __uint_as_float(w[k] << 16);
    f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}
RDP_DEV uint4 pack8f(const float* f) {
  uint4 v;
  v.x = pack2bf(f[0], f[1]);
  v.y = pack2bf(f[2], f[3]);
  v.z = pack2bf(f[4], f[5]);
  v.w = pack2bf(f[6], f[7]);
  return v;
}

__global__ void maxpool2_fwd_kernel(const u16* __restrict__ x, int xpitch, u16* __restrict__ out, int opitch, int N,
                                    int H, int W, int C) {
  const int Ho = H / 2, Wo = W / 2, CG = C >> 3;
  const long total = (long)N * Ho * Wo * CG;
  for (long it = blockIdx.x * (long)blockDim.x + threadIdx.x; it < total; it += (long)gridDim.x * blockDim.x) {
    const int g = it % CG;
    const long po = it / CG;
    const int wo = po % Wo;
    const long t = po / Wo;
    const int ho = t % Ho, n = t / Ho;
    const long p00 = ((long)n * H + 2 * ho) * W + 2 * wo;
    const int c = g * 8;
    float v[4][8];
    unpack8f(*(const uint4*)(x + p00 * xpitch + c), v[0]);
    unpack8f(*(const uint4*)(x + (p00 + 1) * xpitch + c), v[1]);
    unpack8f(*(const uint4*)(x + (p00 + W) * xpitch + c), v[2]);
    unpack8f(*(const uint4*)(x + (p00 + W + 1) * xpitch + c), v[3]);
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float m = v[0][k];
#pragma unroll
      for (int q = 1; q < 4; ++q)
        if (v[q][k] > m || isnan(v[q][k])) m = v[q][k];
      o[k] = m;
    }
    *(uint4*)(out + po * opitch + c) = pack8f(o);
  }
}

// dx[2x2 window] = (argmax ? dp : 0) + dskip ; pixels outside every window get dskip only.
__global__ void maxpool2_bwd_kernel(const u16* __restrict__ dp, int dppitch, const u16* __restrict__ x, int xpitch,
                                    const u16* __restrict__ dskip, int dspitch, u16* __restrict__ dx, int dxpitch,
                                    int N, int H, int W, int C) {
  const int Ho = H / 2, Wo = W / 2, CG = C >> 3;
  const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;  // windows covering every pixel
  const long total = (long)N * Hc * Wc * CG;
  for (long it = blockIdx.x * (long)blockDim.x + threadIdx.x; it < total; it += (long)gridDim.x * blockDim.x) {
    const int g = it % CG;
    const long pw = it / CG;
    const int wc = pw % Wc;
    const long t = pw / Wc;
    const int hc = t % Hc, n = t / Hc;
    const int c = g * 8;
    const bool pooled = hc < Ho && wc < Wo;
    float v[4][8], d[8], o[4][8];
    int idx[8];
    if (pooled) {
      const long p00 = ((long)n * H + 2 * hc) * W + 2 * wc;
      unpack8f(*(const uint4*)(x + p00 * xpitch + c), v[0]);
      unpack8f(*(const uint4*)(x + (p00 + 1) * xpitch + c), v[1]);
      unpack8f(*(const uint4*)(x + (p00 + W) * xpitch + c), v[2]);
      unpack8f(*(const uint4*)(x + (p00 + W + 1) * xpitch + c), v[3]);
      const long po = ((long)n * Ho + hc) * Wo + wc;
      unpack8f(*(const uint4*)(dp + po * dppitch + c), d);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float m = v[0][k];
        int id = 0;
#pragma unroll
        for (int q = 1; q < 4; ++q)
          if (v[q][k] > m || isnan(v[q][k])) { m = v[q][k]; id = q; }
        idx[k] = id;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int hh = 2 * hc + (q >> 1), ww = 2 * wc + (q & 1);
      if (hh >= H || ww >= W) continue;
      const long p = ((long)n * H + hh) * W + ww;
      float s[8];
      if (dskip) unpack8f(*(const uint4*)(dskip + p * dspitch + c), s);
      else {
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] = 0.f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) o[q][k] = s[k] + ((pooled && idx[k] == q) ? d[k] : 0.f);
      *(uint4*)(dx + p * dxpitch + c) = pack8f(o[q]);
    }
  }
}

// ---- BN/ReLU <-> maxpool fusions at the encoder's Down boundaries (training) ----
// Forward: the last conv of each encoder DoubleConv feeds both the skip connection and MaxPool2d
// (segmentation_model.py:47,110-114). One pass reads its pre-BN output y once and writes the skip
// activation a = relu(y*scale + shift) AND the pooled tensor (the standalone pool re-read a).
// Backward: the pool's backward (+ skip gradient) is that layer's activation gradient, so the BN
// backward reduction (sum g, sum g*xhat over the ReLU mask) runs in the same pass on the values it
// just produced instead of re-reading them. Each thread owns one 8-channel group for the launch
// (coefficients in registers) and walks 2x2 windows with a grid stride; C is a power of two.
RDP_DEV void ld8f(const float* p, float* f) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

__global__ __launch_bounds__(256) void bn_relu_apply_pool_kernel(const u16* __restrict__ y, int ypitch,
                                                                 u16* __restrict__ a, int apitch,
                                                                 u16* __restrict__ pool, int ppitch,
                                                                 const float* __restrict__ coef, int N, int H, int W,
                                                                 int C) {
  const int CG = C >> 3, RPB = 256 / CG;
  const int g = threadIdx.x & (CG - 1), r = threadIdx.x / CG;
  const int c = g * 8;
  float ss[8], hh[8];
  ld8f(coef + 2 * C + c, ss);
  ld8f(coef + 3 * C + c, hh);
  const int Ho = H / 2, Wo = W / 2, Hc = (H + 1) / 2, Wc = (W + 1) / 2;
  const int nwin = N * Hc * Wc;
  for (int wi = blockIdx.x * RPB + r; wi < nwin; wi += gridDim.x * RPB) {
    const int wc = wi % Wc, t = wi / Wc;
    const int hc = t % Hc, n = t / Hc;
    uint4 v[4];
    bool ok[4];
    long px[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int h = 2 * hc + (q >> 1), w = 2 * wc + (q & 1);
      ok[q] = h < H && w < W;
      px[q] = ((long)n * H + h) * W + w;
      if (ok[q]) v[q] = *(const uint4*)(y + px[q] * ypitch + c);
    }
    float av[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!ok[q]) continue;
      float f[8];
      unpack8f(v[q], f);
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = fmaxf(fmaf(f[k], ss[k], hh[k]), 0.f);
      const uint4 o = pack8f(f);
      if (a) *(uint4*)(a + px[q] * apitch + c) = o;  // a == nullptr: pool only (the caller writes a elsewhere)
      unpack8f(o, av[q]);  // the pool sees exactly the stored (bf16) activation
    }
    if (hc < Ho && wc < Wo) {
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float m = av[0][k];
#pragma unroll
        for (int q = 1; q < 4; ++q)
          if (av[q][k] > m || isnan(av[q][k])) m = av[q][k];
        o[k] = m;
      }
      *(uint4*)(pool + (((long)n * Ho + hc) * Wo + wc) * ppitch + c) = pack8f(o);
    }
  }
}

// dx = maxpool_bwd(dp) (+ dskip), then partial[blk] = [sum_g | sum_g*xhat] per channel with
// g = dx * (y*scale + shift > 0), xhat = (y - mean) * invstd (bn_relu_bwd_reduce's partial format).
// The pool's argmax comes from the activation recomputed from y (read anyway for the reduction), so
// the stored activation is not read at all.
__global__ __launch_bounds__(256) void maxpool2_bwd_bn_reduce_kernel(
    const u16* __restrict__ dp, int dppitch, const u16* __restrict__ dskip,
    int dspitch, u16* __restrict__ dx, int dxpitch, const u16* __restrict__ y, int ypitch,
    const float* __restrict__ coef, int N, int H, int W, int C, float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float sred[];  // [rows][C][2]
  const int CG = C >> 3, RPB = 256 / CG;
  const int g = threadIdx.x & (CG - 1), r = threadIdx.x / CG;
  const int c = g * 8;
  float mean[8], inv[8], ss[8], hh[8];
  ld8f(coef + c, mean);
  ld8f(coef + C + c, inv);
  ld8f(coef + 2 * C + c, ss);
  ld8f(coef + 3 * C + c, hh);
  float sg[8], sgx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { sg[k] = 0.f; sgx[k] = 0.f; }
  const int Ho = H / 2, Wo = W / 2, Hc = (H + 1) / 2, Wc = (W + 1) / 2;
  const int nwin = N * Hc * Wc;
  for (int wi = blockIdx.x * RPB + r; wi < nwin; wi += gridDim.x * RPB) {
    const int wc = wi % Wc, t = wi / Wc;
    const int hc = t % Hc, n = t / Hc;
    const bool pooled = hc < Ho && wc < Wo;
    bool ok[4];
    long px[4];
    uint4 vs[4], vy[4], vd;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int h = 2 * hc + (q >> 1), w = 2 * wc + (q & 1);
      ok[q] = h < H && w < W;
      px[q] = ((long)n * H + h) * W + w;
      if (ok[q]) {
        vy[q] = *(const uint4*)(y + px[q] * ypitch + c);
        vs[q] = dskip ? *(const uint4*)(dskip + px[q] * dspitch + c) : make_uint4(0, 0, 0, 0);
      }
    }
    if (pooled) vd = *(const uint4*)(dp + (((long)n * Ho + hc) * Wo + wc) * dppitch + c);
    int idx[8];
    float d[8];
    if (pooled) {
      // the forward pool's inputs, recomputed bit-exactly from y (bn_relu_apply_pool's arithmetic)
      // instead of re-reading the stored activation
      float v[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float f[8];
        unpack8f(vy[q], f);
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] = fmaxf(fmaf(f[k], ss[k], hh[k]), 0.f);
        unpack8f(pack8f(f), v[q]);
      }
      unpack8f(vd, d);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float m = v[0][k];
        int id = 0;
#pragma unroll
        for (int q = 1; q < 4; ++q)
          if (v[q][k] > m || isnan(v[q][k])) { m = v[q][k]; id = q; }
        idx[k] = id;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!ok[q]) continue;
      float sk[8], o[8], fy[8];
      unpack8f(vs[q], sk);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = sk[k] + ((pooled && idx[k] == q) ? d[k] : 0.f);
      const uint4 ov = pack8f(o);
      *(uint4*)(dx + px[q] * dxpitch + c) = ov;
      unpack8f(ov, o);  // reduce the stored (bf16) gradient, as the standalone reduce would
      unpack8f(vy[q], fy);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float gg = fmaf(fy[k], ss[k], hh[k]) > 0.f ? o[k] : 0.f;
        sg[k] += gg;
        sgx[k] += gg * (fy[k] - mean[k]) * inv[k];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sred[(r * C + c + k) * 2] = sg[k];
    sred[(r * C + c + k) * 2 + 1] = sgx[k];
  }
  __syncthreads();
  for (int cc = threadIdx.x; cc < C; cc += 256) {
    float a0 = 0.f, a1 = 0.f;
    for (int q = 0; q < RPB; ++q) { a0 += sred[(q * C + cc) * 2]; a1 += sred[(q * C + cc) * 2 + 1]; }
    partial[(size_t)blockIdx.x * 2 * C + cc] = a0;
    partial[(size_t)blockIdx.x * 2 * C + C + cc] = a1;
  }
}

struct UpGeom {
  int N, hin, win, Hout, Wout, oy, ox, C;
  float rh, rw;
};

RDP_DEV void up_src(int u, int in, float r, int& i0, int& i1, float& l1) {
  const float s = r * (float)u;
  i0 = (int)s;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = s - (float)i0;
}

// Row-blocked bilinear x2 (align_corners=True). One work item = one output (fwd) / input-gradient
// (bwd) image row segment of 256 (pixel, 8-channel group) pairs: the row's source rows and weights
// are block-uniform (scalar), channel groups are a power of two, so the per-thread indexing is shifts
// and masks (no 64-bit division), and every access is a 16-B, line-coalesced vector.
// coef != nullptr: x is the producing layer's PRE-BN output; its training BN + ReLU (coef =
// [mean|invstd|scale|shift]) is applied to each tap and rounded to bf16 exactly as bn_relu_apply would
// store it, so the post-activation tensor of the layer below every Up block is never materialised.
RDP_DEV void bn_relu8(float* v, const float* sc, const float* sh) {
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = bf2f(f2bf(fmaxf(fmaf(v[k], sc[k], sh[k]), 0.f)));
}

// R = 1 (too few rows for bands, e.g. batch-1 serving): one output row per work item, 4 taps per output.
__global__ __launch_bounds__(256) void upsample2_fwd_taps_kernel(const u16* __restrict__ x, int xpitch,
                                                                 u16* __restrict__ out, int opitch, UpGeom g, int lcg,
                                                                 int nchunk, const float* __restrict__ coef) {
  const int CG = 1 << lcg;
  const int items = g.N * g.Hout * nchunk;
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int row = it / nchunk, q = it - row * nchunk;
    const int n = row / g.Hout, Y = row - n * g.Hout;
    const int t = q * 256 + threadIdx.x;
    const int X = t >> lcg, c = (t & (CG - 1)) * 8;
    if (X >= g.Wout) continue;
    const int uy = Y - g.oy, ux = X - g.ox;
    float o[8];
    if (uy < 0 || ux < 0 || uy >= 2 * g.hin || ux >= 2 * g.win) {
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = 0.f;
    } else {
      int y0, y1, x0, x1;
      float ly, lx;
      up_src(uy, g.hin, g.rh, y0, y1, ly);
      up_src(ux, g.win, g.rw, x0, x1, lx);
      const long base = (long)n * g.hin;
      float a[8], b[8], cc[8], d[8];
      unpack8f(*(const uint4*)(x + ((base + y0) * g.win + x0) * xpitch + c), a);
      unpack8f(*(const uint4*)(x + ((base + y0) * g.win + x1) * xpitch + c), b);
      unpack8f(*(const uint4*)(x + ((base + y1) * g.win + x0) * xpitch + c), cc);
      unpack8f(*(const uint4*)(x + ((base + y1) * g.win + x1) * xpitch + c), d);
      if (coef) {
        float sc[8], sh[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { sc[k] = coef[2 * g.C + c + k]; sh[k] = coef[3 * g.C + c + k]; }
        bn_relu8(a, sc, sh); bn_relu8(b, sc, sh); bn_relu8(cc, sc, sh); bn_relu8(d, sc, sh);
      }
      const float hy = 1.f - ly, hx = 1.f - lx;
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = hy * (hx * a[k] + lx * b[k]) + ly * (hx * cc[k] + lx * d[k]);
    }
    *(uint4*)(out + ((long)row * g.Wout + X) * opitch + c) = pack8f(o);
  }
}

// One work item = a band of R output rows x 256 (pixel, 8-channel group) columns; each thread walks
// its column down the band. The interpolation is evaluated in PyTorch's order, horizontal blend of each
// source row first, h = hx*x[y][x0] + lx*x[y][x1], then o = hy*h[y0] + ly*h[y1]: the source-row
// blends are kept in registers while the row pair slides down (y0/y1 advance by at most one per
// output row), so a band of R rows loads ~R/2+1 source-row pairs instead of 4 taps per output.
RDP_DEV void up_hrow(const u16* __restrict__ x, long rowbase, int x0, int x1, int xpitch, int c, float hx,
                     float lx, const float* __restrict__ coef, int C, float* h) {
  float a[8], b[8];
  unpack8f(*(const uint4*)(x + (rowbase + x0) * xpitch + c), a);
  unpack8f(*(const uint4*)(x + (rowbase + x1) * xpitch + c), b);
  if (coef) {
    float sc[8], sh[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { sc[k] = coef[2 * C + c + k]; sh[k] = coef[3 * C + c + k]; }
    bn_relu8(a, sc, sh); bn_relu8(b, sc, sh);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = hx * a[k] + lx * b[k];
}

__global__ __launch_bounds__(256) void upsample2_fwd_kernel(const u16* __restrict__ x, int xpitch,
                                                            u16* __restrict__ out, int opitch, UpGeom g, int lcg,
                                                            int nchunk, int R, const float* __restrict__ coef) {
  const int CG = 1 << lcg;
  const int nband = (g.Hout + R - 1) / R;
  const int items = g.N * nband * nchunk;
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int band = it / nchunk, q = it - band * nchunk;
    const int n = band / nband, Yb = (band - n * nband) * R;
    const int t = q * 256 + threadIdx.x;
    const int X = t >> lcg, c = (t & (CG - 1)) * 8;
    if (X >= g.Wout) continue;
    const int ux = X - g.ox;
    const bool xin = ux >= 0 && ux < 2 * g.win;
    int x0 = 0, x1 = 0;
    float lx = 0.f;
    if (xin) up_src(ux, g.win, g.rw, x0, x1, lx);
    const float hx = 1.f - lx;
    const long base = (long)n * g.hin;
    float h0[8], h1[8];
    int r0 = -1, r1 = -1;  // source rows held in h0 / h1
    const int Ye = min(Yb + R, g.Hout);
    for (int Y = Yb; Y < Ye; ++Y) {
      const int uy = Y - g.oy;
      float o[8];
      if (!xin || uy < 0 || uy >= 2 * g.hin) {
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = 0.f;
      } else {
        int y0, y1;
        float ly;
        up_src(uy, g.hin, g.rh, y0, y1, ly);
        if (y0 != r0) {
          if (y0 == r1) {
#pragma unroll
            for (int k = 0; k < 8; ++k) h0[k] = h1[k];
          } else {
            up_hrow(x, (base + y0) * g.win, x0, x1, xpitch, c, hx, lx, coef, g.C, h0);
          }
          r0 = y0;
        }
        if (y1 != r1) {
          if (y1 == r0) {
#pragma unroll
            for (int k = 0; k < 8; ++k) h1[k] = h0[k];
          } else {
            up_hrow(x, (base + y1) * g.win, x0, x1, xpitch, c, hx, lx, coef, g.C, h1);
          }
          r1 = y1;
        }
        const float hy = 1.f - ly;
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = hy * h0[k] + ly * h1[k];
      }
      *(uint4*)(out + (((long)n * g.Hout + Y) * g.Wout + X) * opitch + c) = pack8f(o);
    }
  }
}

RDP_DEV float up_weight(int u, int in, float r, int i) {
  int i0, i1;
  float l1;
  up_src(u, in, r, i0, i1, l1);
  return (i0 == i ? 1.f - l1 : 0.f) + (i1 == i ? l1 : 0.f);
}

// dx[n][i][j] = sum_{uy,ux} w(uy,i) w(ux,j) dout[n][uy+oy][ux+ox]. With r = (in-1)/(2in-1) < 1/2,
// a nonzero w(u,i) needs floor(u*r) in {i-1, i}, which holds only for u in [2i-1, 2i+2]: a fixed
// 4x4 window, evaluated separably: h(uy) = sum_ux w(ux,j) dout[uy][ux] (4 taps, clamped address,
// weight 0 outside the image), dx = sum_uy w(uy,i) h(uy) in ascending uy. One work item = a band of R
// input-gradient rows x 256 (pixel, 8-channel group) columns; walking down the band, rows 2i+1, 2i+2
// of i are rows 2i'-1, 2i' of i' = i+1, so each row after the first loads 2 new h rows (8 taps)
// instead of 16.
// BNR: the consumer's training-BN backward reduction of g = bf16(dx) * relu'(y*scale+shift) is
// accumulated on the fly (bn_relu_bwd_reduce layout, one partial row per block), so dx is never
// re-read for it.
RDP_DEV void up_hsum(const u16* __restrict__ dout, long ro, const int* xo, const float* wx, int dpitch, int c,
                     float* h) {
  uint4 v[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) v[b] = *(const uint4*)(dout + (ro + xo[b]) * dpitch + c);
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = 0.f;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    float d[8];
    unpack8f(v[b], d);
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = fmaf(wx[b], d[k], h[k]);
  }
}

template <bool BNR>
__global__ __launch_bounds__(256) void upsample2_bwd_kernel(const u16* __restrict__ dout, int dpitch,
                                                            u16* __restrict__ dx, int xpitch, UpGeom g, int lcg,
                                                            int nchunk, int R, const u16* __restrict__ y,
                                                            int ypitch, const float* __restrict__ coef,
                                                            float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float sred[];  // BNR: [256 / CG][C][2]
  const int CG = 1 << lcg;
  const int uh = 2 * g.hin, uw = 2 * g.win;
  const int c = (threadIdx.x & (CG - 1)) * 8;
  float mean[8], inv[8], ss[8], hh[8], sg[8], sgx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sg[k] = 0.f;
    sgx[k] = 0.f;
    if (BNR) {
      mean[k] = coef[c + k];
      inv[k] = coef[g.C + c + k];
      ss[k] = coef[2 * g.C + c + k];
      hh[k] = coef[3 * g.C + c + k];
    }
  }
  const int nband = (g.hin + R - 1) / R;
  const int items = g.N * nband * nchunk;
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int band = it / nchunk, q = it - band * nchunk;
    const int n = band / nband, ib = (band - n * nband) * R, ie = min(ib + R, g.hin);
    const int j = (q * 256 + threadIdx.x) >> lcg;
    if (j >= g.win) continue;
    float wx[4];
    int xo[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ux = 2 * j - 1 + t, X = ux + g.ox;
      const bool okx = ux >= 0 && ux < uw && X >= 0 && X < g.Wout;
      wx[t] = okx ? up_weight(ux, g.win, g.rw, j) : 0.f;
      xo[t] = okx ? X : 0;
    }
    auto rowoff = [&](int uy) {
      const int Y = uy + g.oy;
      const bool oky = uy >= 0 && uy < uh && Y >= 0 && Y < g.Hout;
      return ((long)n * g.Hout + (oky ? Y : 0)) * g.Wout;
    };
    float h0[8], h1[8], h2[8], h3[8];  // h(2i-1) .. h(2i+2)
    up_hsum(dout, rowoff(2 * ib - 1), xo, wx, dpitch, c, h2);
    up_hsum(dout, rowoff(2 * ib), xo, wx, dpitch, c, h3);
    for (int i = ib; i < ie; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) { h0[k] = h2[k]; h1[k] = h3[k]; }
      up_hsum(dout, rowoff(2 * i + 1), xo, wx, dpitch, c, h2);
      up_hsum(dout, rowoff(2 * i + 2), xo, wx, dpitch, c, h3);
      float wy[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int uy = 2 * i - 1 + t, Y = uy + g.oy;
        const bool oky = uy >= 0 && uy < uh && Y >= 0 && Y < g.Hout;
        wy[t] = oky ? up_weight(uy, g.hin, g.rh, i) : 0.f;
      }
      float acc[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        acc[k] = wy[0] * h0[k];
        acc[k] = fmaf(wy[1], h1[k], acc[k]);
        acc[k] = fmaf(wy[2], h2[k], acc[k]);
        acc[k] = fmaf(wy[3], h3[k], acc[k]);
      }
      const int row = n * g.hin + i;
      const long p = (long)row * g.win + j;
      const uint4 o = pack8f(acc);
      *(uint4*)(dx + p * xpitch + c) = o;
      if (BNR) {
        float fg[8], fy[8];
        unpack8f(o, fg);
        unpack8f(*(const uint4*)(y + p * ypitch + c), fy);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float gg = fmaf(fy[k], ss[k], hh[k]) > 0.f ? fg[k] : 0.f;
          sg[k] += gg;
          sgx[k] += gg * (fy[k] - mean[k]) * inv[k];
        }
      }
    }
  }
  if (BNR) {
    const int RPB = 256 >> lcg, r = threadIdx.x >> lcg;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sred[(r * g.C + c + k) * 2] = sg[k];
      sred[(r * g.C + c + k) * 2 + 1] = sgx[k];
    }
    __syncthreads();
    for (int cc = threadIdx.x; cc < g.C; cc += 256) {
      float a0 = 0.f, a1 = 0.f;
      for (int qq = 0; qq < RPB; ++qq) { a0 += sred[(qq * g.C + cc) * 2]; a1 += sred[(qq * g.C + cc) * 2 + 1]; }
      partial[(size_t)blockIdx.x * 2 * g.C + cc] = a0;
      partial[(size_t)blockIdx.x * 2 * g.C + g.C + cc] = a1;
    }
  }
}

static int gridN(long items) {
  long g = (items + 255) / 256;
  return (int)std::max<long>(1, std::min<long>(g, 4096));
}
static float ac_scale(int in, int out) { return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f; }

// ---- ConvTranspose2d(k=2, s=2) around a 1x1 GEMM (Up block of the transposed decoder) ----
// Reference op: nn.ConvTranspose2d(cin, cin//2, 2, stride=2) + F.pad in Up.forward
// (/root/reference/pkg/segmentation_model.py:64,68-74). The GEMM yT[px][(dh*2+dw)*C + c] =
// sum_ci x[px][ci] W[ci][c][dh][dw] runs on the conv kernel (taps = 1); these kernels move the
// 2x2 sub-pixels into place (+ bias, zero pad) and back.
struct UpTGeom {
  int N, h, w, H2, W2, oy, ox, C;
};

// u[n][y][x][c..c+7] = yT[n][(y-oy)/2][(x-ox)/2][((y-oy)&1)*2 + ((x-ox)&1)][c..] + bias, 0 outside
__global__ void upT_shuffle_kernel(const u16* __restrict__ yT, int ypitch, const float* __restrict__ bias,
                                   u16* __restrict__ u, int upitch, UpTGeom g) {
  const int CG = g.C >> 3;
  const long total = (long)g.N * g.H2 * g.W2 * CG;
  for (long it = blockIdx.x * (long)blockDim.x + threadIdx.x; it < total; it += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(it % CG);
    const long pix = it / CG;
    const int x = (int)(pix % g.W2);
    const long t = pix / g.W2;
    const int y = (int)(t % g.H2), n = (int)(t / g.H2);
    const int hy = y - g.oy, wx = x - g.ox;
    const int c = cg * 8;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (hy >= 0 && hy < 2 * g.h && wx >= 0 && wx < 2 * g.w) {
      const long src = ((long)n * g.h + (hy >> 1)) * g.w + (wx >> 1);
      const int j = ((hy & 1) * 2 + (wx & 1)) * g.C + c;
      float f[8];
      unpack8f(*(const uint4*)(yT + src * ypitch + j), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] += bias[c + k];
      v = pack8f(f);
    }
    *(uint4*)(u + pix * upitch + c) = v;
  }
}

// dyT[n][h][w][(dh*2+dw)*C + c] = du[n][2h+dh+oy][2w+dw+ox][c]
__global__ void upT_unshuffle_kernel(const u16* __restrict__ du, int dpitch, u16* __restrict__ dyT, int ypitch,
                                     UpTGeom g) {
  const int CG4 = (4 * g.C) >> 3;
  const long total = (long)g.N * g.h * g.w * CG4;
  for (long it = blockIdx.x * (long)blockDim.x + threadIdx.x; it < total; it += (long)gridDim.x * blockDim.x) {
    const int jg = (int)(it % CG4);
    const long pix = it / CG4;
    const int ww = (int)(pix % g.w);
    const long t = pix / g.w;
    const int hh = (int)(t % g.h), n = (int)(t / g.h);
    const int j = jg * 8, sub = j / g.C, c = j - sub * g.C;
    const int y = 2 * hh + (sub >> 1) + g.oy, x = 2 * ww + (sub & 1) + g.ox;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (y >= 0 && y < g.H2 && x >= 0 && x < g.W2) v = *(const uint4*)(du + (((long)n * g.H2 + y) * g.W2 + x) * dpitch + c);
    *(uint4*)(dyT + pix * ypitch + j) = v;
  }
}

// Bias gradient: out[c] (+)= sum_rows sum_{g < groups} x[row][g*C + c]  (x bf16 [M][groups*C]).
// Stage 1: per-block partial column sums (thread = fixed 8-column group); stage 2: fold + write.
__global__ __launch_bounds__(256) void colsum_bf16_kernel(const u16* __restrict__ x, int pitch, long M, int K,
                                                          float* __restrict__ partial) {
  extern __shared__ float sred2[];
  const int CG = K >> 3, RPB = 256 / CG;  // K = groups*C, power of two <= 2048
  const int g = threadIdx.x % CG, r = threadIdx.x / CG;
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  if (r < RPB)
    for (long p = blockIdx.x * (long)RPB + r; p < M; p += (long)gridDim.x * RPB) {
      float f[8];
      unpack8f(*(const uint4*)(x + p * pitch + g * 8), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += f[k];
    }
  if (r < RPB)
#pragma unroll
    for (int k = 0; k < 8; ++k) sred2[r * K + g * 8 + k] = acc[k];
  __syncthreads();
  for (int cc = threadIdx.x; cc < K; cc += 256) {
    float s = 0.f;
    for (int q = 0; q < RPB; ++q) s += sred2[q * K + cc];
    partial[(long)blockIdx.x * K + cc] = s;
  }
}
// Stage 2a: the (block, group) partial rows folded in FOLD_RB row chunks: block (channel block of 64,
// chunk) = 4 waves striding over the chunk's rows (coalesced 256 B row reads, 4 loads in flight per
// lane, fp64), fixed-order LDS fold -> part2[chunk][c]. Stage 2b sums the chunks in order
// (deterministic). One block per 64 channels walking every row took 83 us per call at nblk 1024
// (bs 64, transposed decoder): latency-bound.
constexpr int FOLD_RB = 32;
__global__ __launch_bounds__(256) void colsum_fold_kernel(const float* __restrict__ partial, int nblk, int K, int groups,
                                                          double* __restrict__ part2) {
  __shared__ double sfold[4][64];
  const int C = K / groups;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  const long rows = (long)nblk * groups;
  const long r0 = rows * blockIdx.y / FOLD_RB, r1 = rows * (blockIdx.y + 1) / FOLD_RB;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (c < C) {
    long q = r0 + ty;
    for (; q + 12 < r1; q += 16) {
      const float v0 = partial[(q / groups) * K + (q % groups) * C + c];
      const float v1 = partial[((q + 4) / groups) * K + ((q + 4) % groups) * C + c];
      const float v2 = partial[((q + 8) / groups) * K + ((q + 8) % groups) * C + c];
      const float v3 = partial[((q + 12) / groups) * K + ((q + 12) % groups) * C + c];
      s0 += v0; s1 += v1; s2 += v2; s3 += v3;
    }
    for (; q < r1; q += 4) s0 += partial[(q / groups) * K + (q % groups) * C + c];
  }
  sfold[ty][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ty == 0 && c < C) part2[(long)blockIdx.y * C + c] = ((sfold[0][tx] + sfold[1][tx]) + sfold[2][tx]) + sfold[3][tx];
}
__global__ __launch_bounds__(256) void colsum_fold2_kernel(const double* __restrict__ part2, int C, float* __restrict__ out,
                                                           int accumulate) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  double t = 0.0;
#pragma unroll
  for (int k = 0; k < FOLD_RB; ++k) t += part2[(long)k * C + c];
  out[c] = accumulate ? out[c] + (float)t : (float)t;
}


extern "C" {
int rdp_maxpool2_fwd(const void* x, int xpitch, void* out, int opitch, int N, int H, int W, int C, hipStream_t s) {
  if (C % 8 || xpitch % 8 || opitch % 8) return -1;
  hipLaunchKernelGGL(maxpool2_fwd_kernel, dim3(gridN((long)N * (H / 2) * (W / 2) * (C / 8))), dim3(256), 0, s,
                     (const u16*)x, xpitch, (u16*)out, opitch, N, H, W, C);
  return 0;
}
int rdp_maxpool2_bwd(const void* dp, int dppitch, const void* x, int xpitch, const void* dskip, int dspitch, void* dx,
                     int dxpitch, int N, int H, int W, int C, hipStream_t s) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(maxpool2_bwd_kernel, dim3(gridN((long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8))), dim3(256),
                     0, s, (const u16*)dp, dppitch, (const u16*)x, xpitch, (const u16*)dskip, dspitch, (u16*)dx,
                     dxpitch, N, H, W, C);
  return 0;
}
static bool pow2c(int C) { return C >= 8 && C <= 2048 && (C & (C - 1)) == 0; }
int rdp_bn_relu_apply_pool(const void* y, int ypitch, void* a, int apitch, void* pool, int ppitch, const float* coef,
                           int N, int H, int W, int C, hipStream_t s) {
  if (!pow2c(C) || ypitch % 8 || apitch % 8 || ppitch % 8) return -1;
  const long rpb = 256 / (C / 8), nwin = (long)N * ((H + 1) / 2) * ((W + 1) / 2);
  // <= 16384 blocks (64/CU): 256^2 x 64 at bs 64 239 -> 219 us, 128^2 x 128 121 -> 116 us vs a 4096 cap
  const int grid = (int)std::max<long>(1, std::min<long>((nwin + rpb - 1) / rpb, 16384));
  hipLaunchKernelGGL(bn_relu_apply_pool_kernel, dim3(grid), dim3(256), 0, s, (const u16*)y, ypitch, (u16*)a, apitch,
                     (u16*)pool, ppitch, coef, N, H, W, C);
  return 0;
}
// returns the number of partial rows written (T for bn_bwd_finalize), -1 if not applicable
// x: the stored activation (pitch check only: the argmax is recomputed from y)
int rdp_maxpool2_bwd_bn_reduce(const void* dp, int dppitch, const void* x, int xpitch, const void* dskip, int dspitch,
                               void* dx, int dxpitch, const void* y, int ypitch, const float* coef, int N, int H, int W,
                               int C, float* partial, int max_blocks, hipStream_t s) {
  if (!pow2c(C) || dppitch % 8 || xpitch % 8 || dspitch % 8 || dxpitch % 8 || ypitch % 8) return -1;
  const long rpb = 256 / (C / 8), nwin = (long)N * ((H + 1) / 2) * ((W + 1) / 2);
  // ~4 windows per thread row: enough bytes in flight, few partial rows for the finalize
  const int grid = (int)std::max<long>(1, std::min<long>((nwin + 4 * rpb - 1) / (4 * rpb), max_blocks));
  const size_t lds = (size_t)rpb * C * 2 * sizeof(float);
  hipLaunchKernelGGL(maxpool2_bwd_bn_reduce_kernel, dim3(grid), dim3(256), lds, s, (const u16*)dp, dppitch,
                     (const u16*)dskip, dspitch, (u16*)dx, dxpitch, (const u16*)y, ypitch, coef,
                     N, H, W, C, partial);
  return grid;
}
static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}
int rdp_upsample2_fwd(const void* x, int xpitch, void* out, int opitch, int N, int hin, int win, int Hout, int Wout,
                      int oy, int ox, int C, const float* coef, hipStream_t s) {
  if (!pow2c(C) || xpitch % 8 || opitch % 8) return -1;
  UpGeom g{N, hin, win, Hout, Wout, oy, ox, C, ac_scale(hin, 2 * hin), ac_scale(win, 2 * win)};
  const int lcg = ilog2(C / 8), nchunk = (int)(((long)Wout * (C / 8) + 255) / 256);
  // band height 8 (128^2 -> 256^2 x 64, bs 64: 196 us with 4 taps per output -> 132 us; 16 rows 139 us),
  // shortened while fewer than 4096 work items (16 waves per CU) would be in flight
  int R = 8;
  while (R > 1 && (long)N * ((Hout + R - 1) / R) * nchunk < 4096) R >>= 1;
  const long items = (long)N * ((Hout + R - 1) / R) * nchunk;
  if (R == 1) {
    hipLaunchKernelGGL(upsample2_fwd_taps_kernel, dim3((int)std::min<long>(items, 8192)), dim3(256), 0, s,
                       (const u16*)x, xpitch, (u16*)out, opitch, g, lcg, nchunk, coef);
    return 0;
  }
  hipLaunchKernelGGL(upsample2_fwd_kernel, dim3((int)std::min<long>(items, 32768)), dim3(256), 0, s, (const u16*)x,
                     xpitch, (u16*)out, opitch, g, lcg, nchunk, R, coef);
  return 0;
}
// y/coef/partial given: fused BN-backward reduction of dx's consumer BN; returns the partial rows
// written (<= max_blocks). Otherwise returns 0.
int rdp_upsample2_bwd(const void* dout, int dpitch, void* dx, int xpitch, int N, int hin, int win, int Hout, int Wout,
                      int oy, int ox, int C, const void* y, int ypitch, const float* coef, float* partial,
                      int max_blocks, hipStream_t s) {
  if (!pow2c(C) || dpitch % 8 || xpitch % 8 || (y && ypitch % 8)) return -1;
  UpGeom g{N, hin, win, Hout, Wout, oy, ox, C, ac_scale(hin, 2 * hin), ac_scale(win, 2 * win)};
  const int lcg = ilog2(C / 8), nchunk = (int)(((long)win * (C / 8) + 255) / 256);
  // band height 4 (256^2 -> 128^2 x 64 + BN reduce, bs 64: 198 us unbanded -> 165 us; 2 rows 171, 8 rows
  // 175), shortened while fewer than 4096 work items would be in flight
  int R = 4;
  while (R > 1 && (long)N * ((hin + R - 1) / R) * nchunk < 4096) R >>= 1;
  const long items = (long)N * ((hin + R - 1) / R) * nchunk;
  if (y) {
    const int grid = (int)std::max<long>(1, std::min<long>(items, max_blocks));
    const size_t lds = (size_t)(256 / (C / 8)) * C * 2 * sizeof(float);
    hipLaunchKernelGGL(upsample2_bwd_kernel<true>, dim3(grid), dim3(256), lds, s, (const u16*)dout, dpitch, (u16*)dx,
                       xpitch, g, lcg, nchunk, R, (const u16*)y, ypitch, coef, partial);
    return grid;
  }
  hipLaunchKernelGGL(upsample2_bwd_kernel<false>, dim3((int)std::min<long>(items, 8192)), dim3(256), 0, s,
                     (const u16*)dout, dpitch, (u16*)dx, xpitch, g, lcg, nchunk, R, (const u16*)nullptr, 0,
                     (const float*)nullptr, (float*)nullptr);
  return 0;
}
int rdp_upT_shuffle(const void* yT, int ypitch, const float* bias, void* u, int upitch, int N, int h, int w, int H2,
                    int W2, int oy, int ox, int C, hipStream_t s) {
  if (C % 8 || ypitch % 8 || upitch % 8) return -1;
  UpTGeom g{N, h, w, H2, W2, oy, ox, C};
  hipLaunchKernelGGL(upT_shuffle_kernel, dim3(gridN((long)N * H2 * W2 * (C / 8))), dim3(256), 0, s, (const u16*)yT,
                     ypitch, bias, (u16*)u, upitch, g);
  return 0;
}
int rdp_upT_unshuffle(const void* du, int dpitch, void* dyT, int ypitch, int N, int h, int w, int H2, int W2, int oy,
                      int ox, int C, hipStream_t s) {
  if (C % 8 || ypitch % 8 || dpitch % 8) return -1;
  UpTGeom g{N, h, w, H2, W2, oy, ox, C};
  hipLaunchKernelGGL(upT_unshuffle_kernel, dim3(gridN((long)N * h * w * (4 * C / 8))), dim3(256), 0, s,
                     (const u16*)du, dpitch, (u16*)dyT, ypitch, g);
  return 0;
}
// partial must hold >= 1024 * K + 2 * FOLD_RB * K / groups floats
int rdp_colsum_bf16(const void* x, int pitch, long M, int K, int groups, float* partial, float* out, int accumulate,
                    hipStream_t s) {
  if (K < 8 || K > 2048 || (K & (K - 1)) || K % groups || pitch % 8) return -1;
  const int rpb = 256 / (K / 8);
  const int nblk = (int)std::max<long>(1, std::min<long>(1024, (M + rpb * 16 - 1) / (rpb * 16)));
  hipLaunchKernelGGL(colsum_bf16_kernel, dim3(nblk), dim3(256), (size_t)rpb * K * sizeof(float), s, (const u16*)x,
                     pitch, M, K, partial);
  const int C = K / groups;
  double* part2 = (double*)(partial + 1024L * K);  // 8-B aligned: K is a power of two >= 8
  hipLaunchKernelGGL(colsum_fold_kernel, dim3((C + 63) / 64, FOLD_RB), dim3(256), 0, s, partial, nblk, K, groups, part2);
  hipLaunchKernelGGL(colsum_fold2_kernel, dim3((C + 255) / 256), dim3(256), 0, s, (const double*)part2, C, out, accumulate);
  return 0;
}
}

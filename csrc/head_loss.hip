// 1x1 output head (64 -> 1, with bias) fused with BCE-with-logits (+ optional soft Dice) loss.
//
// Reference: OutConv = nn.Conv2d(64, n_classes, 1) (/root/reference/pkg/segmentation_model.py:78-84),
// criterion = nn.BCEWithLogitsLoss() mean reduction (scripts/train_segmenter.py:145,161).
// The Dice term is the north-star "BCE-Dice" head (BASELINE.json), off by default.
//
// head_fwd: logits[p] = sum_c a[p][c]*w[c] + b; per-block partials of
//   {sum bce, sum sigmoid*t, sum sigmoid, sum t}  (bce = max(x,0) - x*t + log1p(exp(-|x|)))
// loss_finalize: loss = mean bce + dice_w * (1 - (2I+eps)/(P+T+eps)) into a device scalar.
// head_bwd: dlogit = (sigmoid(x)-t)/M + dice_w * d(dice)/dx; da[p][c] = dlogit*w[c] (bf16);
//   per-block partials of dW (64) and db.
// 8 lanes per pixel (16 B each = 8 channels), so every access is a full 128-B line per pixel.
#include "common.h"
#include <algorithm>

#define HEAD_C 64
#define HPX 4  // pixels in flight per 8-lane group in the streaming head kernels

RDP_DEV void unpack8h(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = __uint_as_float(w[k] << 16);
    f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}

RDP_DEV float dot8(const uint4& v, const float* w) {
  float f[8];
  unpack8h(v, f);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s = fmaf(f[k], w[k], s);
  return s;
}

RDP_DEV float bfround(float f) { return __uint_as_float(((uint32_t)f2bf(f)) << 16); }

RDP_DEV float sum8lanes(float v) {  // reduce across the 8 lanes of a pixel group
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}

// BN = true (training): `a` holds the last conv's PRE-BN output y and coef its BN coefficients
// [mean | invstd | scale | shift] (64 each); the head applies a = bf16(relu(y*scale + shift)) itself,
// so that activation is never written or re-read (up4.conv.double_conv.3 -> outc).
RDP_DEV uint4 bn_relu8(const uint4& v, const float* ss, const float* hh) {
  float f[8];
  unpack8h(v, f);
  uint4 o;
  o.x = pack2bf(fmaxf(fmaf(f[0], ss[0], hh[0]), 0.f), fmaxf(fmaf(f[1], ss[1], hh[1]), 0.f));
  o.y = pack2bf(fmaxf(fmaf(f[2], ss[2], hh[2]), 0.f), fmaxf(fmaf(f[3], ss[3], hh[3]), 0.f));
  o.z = pack2bf(fmaxf(fmaf(f[4], ss[4], hh[4]), 0.f), fmaxf(fmaf(f[5], ss[5], hh[5]), 0.f));
  o.w = pack2bf(fmaxf(fmaf(f[6], ss[6], hh[6]), 0.f), fmaxf(fmaf(f[7], ss[7], hh[7]), 0.f));
  return o;
}

// GRAD (training, BN-fused, BCE only -- d loss / d logit is then local, (sigmoid(x) - t) / M): the
// forward pass also produces everything head_bwd_kernel<true> would, from the same read of y: head
// weight/bias gradient partials gpart[blk][65] and the last conv's BN-backward partials
// bnpart[blk][128]. The backward then only finalizes (no second pass over y).
template <bool BN, bool GRAD>
__global__ __launch_bounds__(256) void head_fwd_kernel(const u16* __restrict__ a, int apitch,
                                                       const float* __restrict__ w, const float* __restrict__ b,
                                                       const float* __restrict__ target, float* __restrict__ logits,
                                                       float* __restrict__ partial, int M,
                                                       const float* __restrict__ coef, float* __restrict__ gpart,
                                                       float* __restrict__ bnpart, float gscale) {
  __shared__ float red[4][4];
  __shared__ float gred[GRAD ? 4 : 1][GRAD ? 3 * HEAD_C + 1 : 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane & 7;
  float wl[8], ss[8], hh[8], mu[8], iv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    wl[k] = w[sub * 8 + k];
    if (BN) { ss[k] = coef[2 * HEAD_C + sub * 8 + k]; hh[k] = coef[3 * HEAD_C + sub * 8 + k]; }
    if (GRAD) { mu[k] = coef[sub * 8 + k]; iv[k] = coef[HEAD_C + sub * 8 + k]; }
  }
  const float bias = b[0];
  const float gs = gscale / (float)M;
  float sb = 0.f, si = 0.f, sp = 0.f, st = 0.f;
  float gw[8], sg[8], sgx[8], gb = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) { gw[k] = 0.f; sg[k] = 0.f; sgx[k] = 0.f; }
  // HPX pixels in flight per 8-lane group (16-B loads issued back to back)
  const long stride = (long)gridDim.x * 32;  // 32 pixel groups per block
  for (long p0 = blockIdx.x * 32l + (threadIdx.x >> 3); p0 < M; p0 += stride * HPX) {
    uint4 v[HPX];
    float tq[HPX];
#pragma unroll
    for (int u = 0; u < HPX; ++u) {
      const long p = p0 + u * stride;
      if (p < M) {
        v[u] = *(const uint4*)(a + (size_t)p * apitch + sub * 8);
        if (GRAD) tq[u] = target[p];
      }
    }
    float xs[HPX];
#pragma unroll
    for (int u = 0; u < HPX; ++u) xs[u] = dot8(BN ? bn_relu8(v[u], ss, hh) : v[u], wl);  // (garbage if p >= M)
#pragma unroll
    for (int u = 0; u < HPX; ++u) xs[u] = sum8lanes(xs[u]);
    if (GRAD) {  // every lane holds the HPX logits: gradients of its 8 channels for all of them
#pragma unroll
      for (int u = 0; u < HPX; ++u) {
        if (p0 + u * stride >= M) break;
        const float x = xs[u] + bias;
        const float e = __expf(-fabsf(x));
        const float sgm = x >= 0.f ? 1.f / (1.f + e) : e / (1.f + e);
        const float dx = (sgm - tq[u]) * gs;
        float fy[8];
        unpack8h(v[u], fy);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float z = fmaf(fy[k], ss[k], hh[k]);
          gw[k] = fmaf(dx, bfround(fmaxf(z, 0.f)), gw[k]);
          const float g = z > 0.f ? bfround(dx * wl[k]) : 0.f;
          sg[k] += g;
          sgx[k] += g * (fy[k] - mu[k]) * iv[k];
        }
        if (sub == 0) gb += dx;
      }
    }
    // lane `sub` finishes pixel `sub`'s logit and loss terms
    float x = xs[0];
#pragma unroll
    for (int u = 1; u < HPX; ++u) x = sub == u ? xs[u] : x;
    x += bias;
    const long p = p0 + sub * stride;
    if (sub < HPX && p < M) {
      logits[p] = x;
      const float t = target[p];
      const float e = __expf(-fabsf(x));
      sb += fmaxf(x, 0.f) - x * t + log1pf(e);
      const float sgm = x >= 0.f ? 1.f / (1.f + e) : e / (1.f + e);
      si += sgm * t;
      sp += sgm;
      st += t;
    }
  }
  sb = wave_sum(sb); si = wave_sum(si); sp = wave_sum(sp); st = wave_sum(st);
  if (lane == 0) { red[wave][0] = sb; red[wave][1] = si; red[wave][2] = sp; red[wave][3] = st; }
  if (GRAD) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // over the 8 pixel groups of the wave sharing `sub`
      float v0 = gw[k], v1 = sg[k], v2 = sgx[k];
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        v0 += __shfl_xor(v0, o, 64);
        v1 += __shfl_xor(v1, o, 64);
        v2 += __shfl_xor(v2, o, 64);
      }
      gw[k] = v0; sg[k] = v1; sgx[k] = v2;
    }
    gb = wave_sum(gb);
    if (lane < 8) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        gred[wave][lane * 8 + k] = gw[k];
        gred[wave][HEAD_C + lane * 8 + k] = sg[k];
        gred[wave][2 * HEAD_C + lane * 8 + k] = sgx[k];
      }
    }
    if (lane == 0) gred[wave][3 * HEAD_C] = gb;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int q = threadIdx.x;
    partial[blockIdx.x * 4 + q] = red[0][q] + red[1][q] + red[2][q] + red[3][q];
  }
  if (GRAD) {
    for (int c = threadIdx.x; c < 3 * HEAD_C + 1; c += 256) {
      const float tot = gred[0][c] + gred[1][c] + gred[2][c] + gred[3][c];
      if (c < HEAD_C) gpart[blockIdx.x * (HEAD_C + 1) + c] = tot;
      else if (c == 3 * HEAD_C) gpart[blockIdx.x * (HEAD_C + 1) + HEAD_C] = tot;
      else bnpart[(size_t)blockIdx.x * 2 * HEAD_C + (c - HEAD_C)] = tot;
    }
  }
}

// sums[0..3] = totals; loss[0] = bce_mean + dice_w * dice
__global__ void loss_finalize_kernel(const float* __restrict__ partial, int T, int M, float dice_w, float dice_eps,
                                     float* __restrict__ sums, float* __restrict__ loss) {
  __shared__ double red[4][64];
  const int q = threadIdx.x >> 6, l = threadIdx.x & 63;  // 256 threads: 4 quantities x 64 lanes
  double s = 0.0;
  for (int t = l; t < T; t += 64) s += (double)partial[t * 4 + q];
  red[q][l] = s;
  __syncthreads();
  if (threadIdx.x < 4) {
    double tot = 0.0;
    for (int k = 0; k < 64; ++k) tot += red[threadIdx.x][k];
    sums[threadIdx.x] = (float)tot;
    red[threadIdx.x][0] = tot;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double bce = red[0][0] / (double)M;
    double L = bce;
    if (dice_w != 0.f) {
      const double dice = 1.0 - (2.0 * red[1][0] + dice_eps) / (red[2][0] + red[3][0] + dice_eps);
      L += dice_w * dice;
    }
    loss[0] = (float)L;
    loss[1] = (float)bce;
  }
}

// d loss / d logit for one pixel (BCE mean + optional soft Dice), times the loss scale
RDP_DEV float head_dlogit(float x, float t, float invM, float dice_w, float I, float den, float dice_eps,
                          float gscale) {
  const float e = __expf(-fabsf(x));
  const float sg = x >= 0.f ? 1.f / (1.f + e) : e / (1.f + e);
  float dx = (sg - t) * invM;
  if (dice_w != 0.f) {
    const float ddp = -(2.f * t * den - (2.f * I + dice_eps)) / (den * den);
    dx += dice_w * ddp * sg * (1.f - sg);
  }
  return dx * gscale;
}

// BN = false: da[p][c] = bf16(dlogit*w[c]) is written for the consumer's BN backward.
// BN = true : `a` is the pre-BN y of the last conv and da is never materialised. The block instead
//   accumulates that BN's backward partials (sum g, sum g*xhat; g = bf16(dlogit*w)*relu'(.)) in the
//   bn_relu_bwd_reduce layout [blk][2][64]; head_bn_bwd_apply recomputes g from the logits.
template <bool BN>
__global__ __launch_bounds__(256) void head_bwd_kernel(const u16* __restrict__ a, int apitch,
                                                       const float* __restrict__ w, const float* __restrict__ logits,
                                                       const float* __restrict__ target, const float* __restrict__ sums,
                                                       u16* __restrict__ da, int dapitch, float* __restrict__ partial,
                                                       int M, float dice_w, float dice_eps, float gscale,
                                                       const float* __restrict__ coef, float* __restrict__ bnpart) {
  __shared__ float red[4][HEAD_C + 1];
  __shared__ float bred[BN ? 4 : 1][BN ? 2 * HEAD_C : 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane & 7;
  float wl[8], mu[8], iv[8], ss[8], hh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    wl[k] = w[sub * 8 + k];
    if (BN) {
      mu[k] = coef[sub * 8 + k];
      iv[k] = coef[HEAD_C + sub * 8 + k];
      ss[k] = coef[2 * HEAD_C + sub * 8 + k];
      hh[k] = coef[3 * HEAD_C + sub * 8 + k];
    }
  }
  const float invM = 1.f / (float)M;
  float I = 0.f, U = 0.f;
  if (dice_w != 0.f) { I = sums[1]; U = sums[2] + sums[3]; }
  const float den = U + dice_eps;
  float gw[8], sg[8], sgx[8], gb = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) { gw[k] = 0.f; sg[k] = 0.f; sgx[k] = 0.f; }
  const long stride = (long)gridDim.x * 32;
  for (long p0 = blockIdx.x * 32l + (threadIdx.x >> 3); p0 < M; p0 += stride * HPX) {
    uint4 vq[HPX];
    float xq[HPX], tq[HPX];
#pragma unroll
    for (int u = 0; u < HPX; ++u) {
      const long p = p0 + u * stride;
      if (p < M) {
        vq[u] = *(const uint4*)(a + (size_t)p * apitch + sub * 8);
        xq[u] = logits[p];
        tq[u] = target[p];
      }
    }
#pragma unroll
    for (int u = 0; u < HPX; ++u) {
      const long p = p0 + u * stride;
      if (p >= M) break;
      const float dx = head_dlogit(xq[u], tq[u], invM, dice_w, I, den, dice_eps, gscale);
      const uint4 vy = vq[u];
      float f[8];
      if (BN) {
        float fy[8];
        unpack8h(vy, fy);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float z = fmaf(fy[k], ss[k], hh[k]);
          f[k] = bfround(fmaxf(z, 0.f));  // the activation the forward head consumed
          const float g = z > 0.f ? bfround(dx * wl[k]) : 0.f;
          sg[k] += g;
          sgx[k] += g * (fy[k] - mu[k]) * iv[k];
        }
      } else {
        unpack8h(vy, f);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) gw[k] = fmaf(dx, f[k], gw[k]);
      if (sub == 0) gb += dx;
      if (!BN) {
        uint4 o;
        o.x = pack2bf(dx * wl[0], dx * wl[1]);
        o.y = pack2bf(dx * wl[2], dx * wl[3]);
        o.z = pack2bf(dx * wl[4], dx * wl[5]);
        o.w = pack2bf(dx * wl[6], dx * wl[7]);
        *(uint4*)(da + (size_t)p * dapitch + sub * 8) = o;
      }
    }
  }
  // reduce over the 8 pixel-groups of the wave that share `sub`
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float v = gw[k];
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    gw[k] = v;
    if (BN) {
      float u = sg[k], q = sgx[k];
      u += __shfl_xor(u, 8, 64);
      u += __shfl_xor(u, 16, 64);
      u += __shfl_xor(u, 32, 64);
      q += __shfl_xor(q, 8, 64);
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      sg[k] = u;
      sgx[k] = q;
    }
  }
  gb = wave_sum(gb);
  if (lane < 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[wave][lane * 8 + k] = gw[k];
      if (BN) {
        bred[wave][lane * 8 + k] = sg[k];
        bred[wave][HEAD_C + lane * 8 + k] = sgx[k];
      }
    }
  }
  if (lane == 0) red[wave][HEAD_C] = gb;
  __syncthreads();
  if (threadIdx.x <= HEAD_C) {
    const int c = threadIdx.x;
    partial[blockIdx.x * (HEAD_C + 1) + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  }
  if (BN && threadIdx.x < 2 * HEAD_C) {
    const int c = threadIdx.x;
    bnpart[(size_t)blockIdx.x * 2 * HEAD_C + c] = bred[0][c] + bred[1][c] + bred[2][c] + bred[3][c];
  }
}

// dy = A*g + B*y + K with g = bf16(dlogit*w)*relu'(y*scale+shift) recomputed per pixel from the
// logits: the last conv's bn_relu_bwd_apply without a materialised da. 4 pixels in flight per
// 8-lane group.
__global__ __launch_bounds__(256) void head_bn_bwd_apply_kernel(const u16* __restrict__ y, int ypitch,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ logits,
                                                                const float* __restrict__ target,
                                                                const float* __restrict__ sums,
                                                                const float* __restrict__ coef,
                                                                const float* __restrict__ coef2,
                                                                u16* __restrict__ dy, int dypitch, int M, float dice_w,
                                                                float dice_eps, float gscale) {
  const int c = (threadIdx.x & 7) * 8;
  float wl[8], ss[8], hh[8], A[8], B[8], K[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    wl[k] = w[c + k];
    ss[k] = coef[2 * HEAD_C + c + k];
    hh[k] = coef[3 * HEAD_C + c + k];
    A[k] = coef2[c + k];
    B[k] = coef2[HEAD_C + c + k];
    K[k] = coef2[2 * HEAD_C + c + k];
  }
  const float invM = 1.f / (float)M;
  float I = 0.f, U = 0.f;
  if (dice_w != 0.f) { I = sums[1]; U = sums[2] + sums[3]; }
  const float den = U + dice_eps;
  constexpr int PX = 4;
  const long stride = (long)gridDim.x * 32;
  for (long p0 = blockIdx.x * 32l + (threadIdx.x >> 3); p0 < M; p0 += stride * PX) {
    uint4 vy[PX];
    float x[PX], t[PX];
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      const long p = p0 + u * stride;
      if (p < M) {
        vy[u] = *(const uint4*)(y + (size_t)p * ypitch + c);
        x[u] = logits[p];
        t[u] = target[p];
      }
    }
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      const long p = p0 + u * stride;
      if (p < M) {
        const float dx = head_dlogit(x[u], t[u], invM, dice_w, I, den, dice_eps, gscale);
        float fy[8], o[8];
        unpack8h(vy[u], fy);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float g = fmaf(fy[k], ss[k], hh[k]) > 0.f ? bfround(dx * wl[k]) : 0.f;
          o[k] = fmaf(A[k], g, fmaf(B[k], fy[k], K[k]));
        }
        uint4 v;
        v.x = pack2bf(o[0], o[1]);
        v.y = pack2bf(o[2], o[3]);
        v.z = pack2bf(o[4], o[5]);
        v.w = pack2bf(o[6], o[7]);
        *(uint4*)(dy + (size_t)p * dypitch + c) = v;
      }
    }
  }
}

// grad[0..63] = dW, grad_b[0] = db: one block per column, 256 threads reduce the T block partials
__global__ void head_grad_finalize_kernel(const float* __restrict__ partial, int T, float* __restrict__ gw,
                                          float* __restrict__ gbias) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  float s = 0.f;
  for (int t = threadIdx.x; t < T; t += 256) s += partial[t * (HEAD_C + 1) + c];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tot = red[0] + red[1] + red[2] + red[3];
    if (c < HEAD_C) gw[c] = tot; else gbias[0] = tot;
  }
}

// serving: logits -> u8 mask at the model resolution (sigmoid(x) > thr  <=>  x > logit(thr))
__global__ void head_mask_kernel(const u16* __restrict__ a, int apitch, const float* __restrict__ w,
                                 const float* __restrict__ b, float logit_thr, uint8_t* __restrict__ mask, int M) {
  const int sub = threadIdx.x & 7;
  float wl[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) wl[k] = w[sub * 8 + k];
  const float bias = b[0];
  for (long p = blockIdx.x * 32l + (threadIdx.x >> 3); p < M; p += (long)gridDim.x * 32) {
    const uint4 v = *(const uint4*)(a + (size_t)p * apitch + sub * 8);
    const float x = sum8lanes(dot8(v, wl)) + bias;
    if (sub == 0) mask[p] = x > logit_thr ? 1 : 0;
  }
}

// (4096-32768 blocks measured slower for head_fwd: 198 -> 213-410 us at 256^2 x 64, bs 64)
static int blocks_for(long M) { return (int)std::max<long>(1, std::min<long>((M + 31) / 32, 2048)); }

extern "C" {
int rdp_head_partial_blocks(long M) { return blocks_for(M); }

// coef != nullptr: `a` is the last conv's pre-BN output; BN+ReLU are applied on the fly.
// gpart/bnpart != nullptr (needs coef, dice_w == 0): also the backward partials (head_fwd_kernel GRAD).
int rdp_head_fwd(const void* a, int apitch, const float* w, const float* b, const float* target, float* logits,
                 float* partial, float* sums, float* loss, int M, float dice_w, float dice_eps, const float* coef,
                 float* gpart, float* bnpart, float gscale, hipStream_t s) {
  if (apitch % 8) return -1;
  if (gpart && (!coef || !bnpart || dice_w != 0.f)) return -1;
  const int nb = blocks_for(M);
  if (gpart)
    hipLaunchKernelGGL((head_fwd_kernel<true, true>), dim3(nb), dim3(256), 0, s, (const u16*)a, apitch, w, b, target,
                       logits, partial, M, coef, gpart, bnpart, gscale);
  else if (coef)
    hipLaunchKernelGGL((head_fwd_kernel<true, false>), dim3(nb), dim3(256), 0, s, (const u16*)a, apitch, w, b, target,
                       logits, partial, M, coef, gpart, bnpart, gscale);
  else
    hipLaunchKernelGGL((head_fwd_kernel<false, false>), dim3(nb), dim3(256), 0, s, (const u16*)a, apitch, w, b,
                       target, logits, partial, M, coef, gpart, bnpart, gscale);
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, s, partial, nb, M, dice_w, dice_eps, sums, loss);
  return nb;
}

// head weight / bias gradient from the [nb][65] partials of a GRAD forward
int rdp_head_grad_finalize(const float* gpart, int M, float* gw, float* gb, hipStream_t s) {
  hipLaunchKernelGGL(head_grad_finalize_kernel, dim3(HEAD_C + 1), dim3(256), 0, s, gpart, blocks_for(M), gw, gb);
  return 0;
}

// coef != nullptr: BN-fused variant (da unused; bnpart receives the BN backward partial rows).
// Returns the number of partial rows.
int rdp_head_bwd(const void* a, int apitch, const float* w, const float* logits, const float* target,
                 const float* sums, void* da, int dapitch, float* partial, float* gw, float* gb, int M, float dice_w,
                 float dice_eps, float gscale, const float* coef, float* bnpart, hipStream_t s) {
  const int nb = blocks_for(M);
  if (coef)
    hipLaunchKernelGGL(head_bwd_kernel<true>, dim3(nb), dim3(256), 0, s, (const u16*)a, apitch, w, logits, target,
                       sums, (u16*)da, dapitch, partial, M, dice_w, dice_eps, gscale, coef, bnpart);
  else
    hipLaunchKernelGGL(head_bwd_kernel<false>, dim3(nb), dim3(256), 0, s, (const u16*)a, apitch, w, logits, target,
                       sums, (u16*)da, dapitch, partial, M, dice_w, dice_eps, gscale, coef, bnpart);
  hipLaunchKernelGGL(head_grad_finalize_kernel, dim3(HEAD_C + 1), dim3(256), 0, s, partial, nb, gw, gb);
  return nb;
}

int rdp_head_bn_bwd_apply(const void* y, int ypitch, const float* w, const float* logits, const float* target,
                          const float* sums, const float* coef, const float* coef2, void* dy, int dypitch, int M,
                          float dice_w, float dice_eps, float gscale, hipStream_t s) {
  if (ypitch % 8 || dypitch % 8) return -1;
  // one 4-pixel step per 8-lane group (M / 128 blocks): 253 -> 196 us at 256^2 x 64, bs 64 (capped at
  // 2048 blocks: 4096 / 8192 measured 283 / 232 us); bs-64 step 19.02 / 18.82 -> 18.82 / 18.82 ms
  const int nb = (int)std::max<long>(1, std::min<long>(((long)M + 127) / 128, 1 << 20));
  hipLaunchKernelGGL(head_bn_bwd_apply_kernel, dim3(nb), dim3(256), 0, s, (const u16*)y, ypitch, w, logits, target,
                     sums, coef, coef2, (u16*)dy, dypitch, M, dice_w, dice_eps, gscale);
  return 0;
}

int rdp_head_mask(const void* a, int apitch, const float* w, const float* b, float logit_thr, void* mask, int M,
                  hipStream_t s) {
  hipLaunchKernelGGL(head_mask_kernel, dim3(blocks_for(M)), dim3(256), 0, s, (const u16*)a, apitch, w, b, logit_thr,
                     (uint8_t*)mask, M);
  return 0;
}
}

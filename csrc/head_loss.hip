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

RDP_DEV float sum8lanes(float v) {  // reduce across the 8 lanes of a pixel group
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}

__global__ __launch_bounds__(256) void head_fwd_kernel(const u16* __restrict__ a, int apitch,
                                                       const float* __restrict__ w, const float* __restrict__ b,
                                                       const float* __restrict__ target, float* __restrict__ logits,
                                                       float* __restrict__ partial, int M) {
  __shared__ float red[4][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane & 7;
  float wl[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) wl[k] = w[sub * 8 + k];
  const float bias = b[0];
  float sb = 0.f, si = 0.f, sp = 0.f, st = 0.f;
  const long groups_per_iter = (long)gridDim.x * 32;  // 32 pixels per block-iteration
  for (long p = blockIdx.x * 32l + (threadIdx.x >> 3); p < M; p += groups_per_iter) {
    const uint4 v = *(const uint4*)(a + (size_t)p * apitch + sub * 8);
    const float x = sum8lanes(dot8(v, wl)) + bias;
    if (sub == 0) {
      logits[p] = x;
      const float t = target[p];
      const float e = __expf(-fabsf(x));
      sb += fmaxf(x, 0.f) - x * t + log1pf(e);
      const float sg = x >= 0.f ? 1.f / (1.f + e) : e / (1.f + e);
      si += sg * t;
      sp += sg;
      st += t;
    }
  }
  sb = wave_sum(sb); si = wave_sum(si); sp = wave_sum(sp); st = wave_sum(st);
  if (lane == 0) { red[wave][0] = sb; red[wave][1] = si; red[wave][2] = sp; red[wave][3] = st; }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int q = threadIdx.x;
    partial[blockIdx.x * 4 + q] = red[0][q] + red[1][q] + red[2][q] + red[3][q];
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

__global__ __launch_bounds__(256) void head_bwd_kernel(const u16* __restrict__ a, int apitch,
                                                       const float* __restrict__ w, const float* __restrict__ logits,
                                                       const float* __restrict__ target, const float* __restrict__ sums,
                                                       u16* __restrict__ da, int dapitch, float* __restrict__ partial,
                                                       int M, float dice_w, float dice_eps, float gscale) {
  __shared__ float red[4][HEAD_C + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane & 7;
  float wl[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) wl[k] = w[sub * 8 + k];
  const float invM = 1.f / (float)M;
  float I = 0.f, U = 0.f;
  if (dice_w != 0.f) { I = sums[1]; U = sums[2] + sums[3]; }
  const float den = U + dice_eps;
  float gw[8], gb = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) gw[k] = 0.f;
  for (long p = blockIdx.x * 32l + (threadIdx.x >> 3); p < M; p += (long)gridDim.x * 32) {
    const float x = logits[p], t = target[p];
    const float e = __expf(-fabsf(x));
    const float sg = x >= 0.f ? 1.f / (1.f + e) : e / (1.f + e);
    float dx = (sg - t) * invM;
    if (dice_w != 0.f) {
      const float ddp = -(2.f * t * den - (2.f * I + dice_eps)) / (den * den);
      dx += dice_w * ddp * sg * (1.f - sg);
    }
    dx *= gscale;
    const uint4 v = *(const uint4*)(a + (size_t)p * apitch + sub * 8);
    float f[8];
    unpack8h(v, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) gw[k] = fmaf(dx, f[k], gw[k]);
    if (sub == 0) gb += dx;
    uint4 o;
    o.x = pack2bf(dx * wl[0], dx * wl[1]);
    o.y = pack2bf(dx * wl[2], dx * wl[3]);
    o.z = pack2bf(dx * wl[4], dx * wl[5]);
    o.w = pack2bf(dx * wl[6], dx * wl[7]);
    *(uint4*)(da + (size_t)p * dapitch + sub * 8) = o;
  }
  // reduce gw over the 8 pixel-groups of the wave that share `sub`
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float v = gw[k];
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    gw[k] = v;
  }
  gb = wave_sum(gb);
  if (lane < 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) red[wave][lane * 8 + k] = gw[k];
  }
  if (lane == 0) red[wave][HEAD_C] = gb;
  __syncthreads();
  if (threadIdx.x <= HEAD_C) {
    const int c = threadIdx.x;
    partial[blockIdx.x * (HEAD_C + 1) + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
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

static int blocks_for(long M) { return (int)std::max<long>(1, std::min<long>((M + 31) / 32, 2048)); }

extern "C" {
int rdp_head_partial_blocks(long M) { return blocks_for(M); }

int rdp_head_fwd(const void* a, int apitch, const float* w, const float* b, const float* target, float* logits,
                 float* partial, float* sums, float* loss, int M, float dice_w, float dice_eps, hipStream_t s) {
  if (apitch % 8) return -1;
  const int nb = blocks_for(M);
  hipLaunchKernelGGL(head_fwd_kernel, dim3(nb), dim3(256), 0, s, (const u16*)a, apitch, w, b, target, logits, partial, M);
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, s, partial, nb, M, dice_w, dice_eps, sums, loss);
  return nb;
}

int rdp_head_bwd(const void* a, int apitch, const float* w, const float* logits, const float* target,
                 const float* sums, void* da, int dapitch, float* partial, float* gw, float* gb, int M, float dice_w,
                 float dice_eps, float gscale, hipStream_t s) {
  const int nb = blocks_for(M);
  hipLaunchKernelGGL(head_bwd_kernel, dim3(nb), dim3(256), 0, s, (const u16*)a, apitch, w, logits, target, sums,
                     (u16*)da, dapitch, partial, M, dice_w, dice_eps, gscale);
  hipLaunchKernelGGL(head_grad_finalize_kernel, dim3(HEAD_C + 1), dim3(256), 0, s, partial, nb, gw, gb);
  return nb;
}

int rdp_head_mask(const void* a, int apitch, const float* w, const float* b, float logit_thr, void* mask, int M,
                  hipStream_t s) {
  hipLaunchKernelGGL(head_mask_kernel, dim3(blocks_for(M)), dim3(256), 0, s, (const u16*)a, apitch, w, b, logit_thr,
                     (uint8_t*)mask, M);
  return 0;
}
}

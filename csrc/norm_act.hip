// Training/eval BatchNorm2d + ReLU kernels on NHWC bf16 activations.
//
// Reference semantics: nn.BatchNorm2d + nn.ReLU(inplace=True) inside DoubleConv
// (/root/reference/pkg/segmentation_model.py:32-36): batch statistics over N*H*W (biased variance
// for normalisation, unbiased for running_var), momentum 0.1, eps 1e-5; eval uses running stats.
//
// Forward statistics arrive as per-M-tile (sum, sumsq) slabs from the conv epilogue
// (conv_igemm.hip); bn_finalize reduces them in fp64, updates running stats and emits the
// per-channel affine (scale, shift) applied by bn_relu_apply. Backward is a two-pass
// reduce (sum g, sum g*xhat) -> finalize (dgamma, dbeta, 3 apply coefficients) -> apply.
#include "common.h"
#include <algorithm>
#include <stdlib.h>

// Stage-1 column reduction: in[T][K] -> out[S][K], S row-chunks reduced by S x ceil(K/64) blocks
// (many CUs, 4 independent accumulators per thread) so the finalize kernels read <= 64 rows.
__global__ void colsum_kernel(const float* __restrict__ in, int T, int K, int rpc, float* __restrict__ out) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + tx;
  const int r0 = blockIdx.y * rpc, r1 = min(T, r0 + rpc);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (col < K) {
    int r = r0 + ty;
    for (; r + 12 < r1; r += 16) {
      a0 += in[(size_t)r * K + col];
      a1 += in[(size_t)(r + 4) * K + col];
      a2 += in[(size_t)(r + 8) * K + col];
      a3 += in[(size_t)(r + 12) * K + col];
    }
    for (; r < r1; r += 4) a0 += in[(size_t)r * K + col];
  }
  red[ty][tx] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (ty == 0 && col < K) out[(size_t)blockIdx.y * K + col] = red[0][tx] + red[1][tx] + red[2][tx] + red[3][tx];
}

// SyncBatchNorm: fold a layer's [T][K] partial rows into K fp64 sums, so one fp64 all-reduce per layer
// carries the rank's statistics (models/unet.py _sync_rows). 64 columns x 16 row groups per block, 4
// loads in flight per thread (one thread per column walked T rows serially: ~150 us per fold).
__global__ __launch_bounds__(1024) void rows_fold_kernel(const float* __restrict__ buf, int T, int K,
                                                         double* __restrict__ out) {
  __shared__ double red[16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + tx;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (col < K) {
    int r = ty;
    for (; r + 48 < T; r += 64) {
      a0 += (double)buf[(size_t)r * K + col];
      a1 += (double)buf[(size_t)(r + 16) * K + col];
      a2 += (double)buf[(size_t)(r + 32) * K + col];
      a3 += (double)buf[(size_t)(r + 48) * K + col];
    }
    for (; r < T; r += 16) a0 += (double)buf[(size_t)r * K + col];
  }
  red[ty][tx] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (ty == 0 && col < K) {
    double t = 0.0;
    for (int g = 0; g < 16; ++g) t += red[g][tx];
    out[col] = t;
  }
}

// the (all-reduced) fp64 sums back as TWO fp32 rows, hi = fp32(sum) and lo = fp32(sum - hi), which the
// finalize kernels add in fp64: the statistics keep ~48 bits instead of fp32's 24 -- E[x^2] - mean^2
// cancels, and one fp32 rounding of the sums moved a small U-Net's bf16 gradients by tens of percent
__global__ void rows_hilo_kernel(const double* __restrict__ in, float* __restrict__ buf, int K) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= K) return;
  const double v = in[col];
  const float hi = (float)v;
  buf[col] = hi;
  buf[K + col] = (float)(v - (double)hi);
}

#define FIN_DIRECT_ROWS 2048
#define FIN_RG 16  // row groups per finalize block (blockDim = 64 * FIN_RG)

// sum over rows t = ty, ty + FIN_RG, ... of p[t][c] and p[t][C + c] (row stride 2C), fp64
// (Measured dead end: 16 rows = 32 loads in flight per thread, tail rows clamped to row T - 1 and
// dropped by a select -- bs 4 step 2.54 -> 2.65 ms, bs 64 20.43 -> 20.59 ms, same box interleaved.)
template <int RG = FIN_RG>
RDP_DEV void fin_rows(const float* __restrict__ p, int T, int C, int c, int ty, double& s, double& q) {
  double s0 = 0.0, s1 = 0.0, q0 = 0.0, q1 = 0.0;
  int t = ty;
  for (; t + 3 * RG < T; t += 4 * RG) {
    const float a0 = p[(size_t)t * 2 * C + c], b0 = p[(size_t)t * 2 * C + C + c];
    const float a1 = p[(size_t)(t + RG) * 2 * C + c], b1 = p[(size_t)(t + RG) * 2 * C + C + c];
    const float a2 = p[(size_t)(t + 2 * RG) * 2 * C + c], b2 = p[(size_t)(t + 2 * RG) * 2 * C + C + c];
    const float a3 = p[(size_t)(t + 3 * RG) * 2 * C + c], b3 = p[(size_t)(t + 3 * RG) * 2 * C + C + c];
    s0 += (double)a0 + (double)a2;
    s1 += (double)a1 + (double)a3;
    q0 += (double)b0 + (double)b2;
    q1 += (double)b1 + (double)b3;
  }
  for (; t < T; t += RG) {
    s0 += (double)p[(size_t)t * 2 * C + c];
    q0 += (double)p[(size_t)t * 2 * C + C + c];
  }
  s = s0 + s1;
  q = q0 + q1;
}

// Measured dead end: one launch per BN pass (each block reduces a row chunk, the last block to
// arrive -- agent-scope fences + a system-scope counter -- runs the finalize) was 7% SLOWER at bs64
// and 40% at bs4 than colsum + finalize: every block's release fence is a full per-XCD L2 writeback
// (buffer_wbl2), far more than the ~6 us kernel boundary it saves.
// reduce [T][K] rows to <= 64 rows in `ws` if needed; returns (pointer, rows)
static const float* shrink_rows(const float* in, int T, int K, float* ws, int& rows, hipStream_t s) {
  // the finalize kernels sum up to FIN_DIRECT_ROWS rows themselves (16 row groups x 64 channels per
  // block, 4 loads in flight per thread): one launch instead of colsum + finalize (bs 4 has 36 BN
  // passes per step, each paying a kernel boundary for the shrink)
  if (T <= FIN_DIRECT_ROWS || ws == nullptr) { rows = T; return in; }
  const int S = 64;
  const int rpc = (T + S - 1) / S;
  hipLaunchKernelGGL(colsum_kernel, dim3((K + 63) / 64, S), dim3(256), 0, s, in, T, K, rpc, ws);
  rows = S;
  return ws;
}

// coef layout: [0:C) mean, [C:2C) invstd, [2C:3C) scale = gamma*invstd, [3C:4C) shift = beta - mean*scale
// CPB channels per block, 1024 / CPB row groups. (16 channels per block -- four times the row groups --
// measured neutral: the ~7 us per finalize is the kernel boundary, not the row walk.)
template <int CPB>
__global__ __launch_bounds__(64 * FIN_RG) void bn_finalize_kernel(const float* __restrict__ stats, int T, int C, double count,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float* __restrict__ rmean, float* __restrict__ rvar, long long* nbt,
                                   float momentum, float eps, float* __restrict__ coef) {
  constexpr int RG = 64 * FIN_RG / CPB;
  __shared__ double red[2][RG][CPB];
  const int tx = threadIdx.x % CPB, ty = threadIdx.x / CPB;
  const int c = blockIdx.x * CPB + tx;
  double s = 0.0, q = 0.0;
  if (c < C) fin_rows<RG>(stats, T, C, c, ty, s, q);
  red[0][ty][tx] = s;
  red[1][ty][tx] = q;
  __syncthreads();
  if (ty == 0 && c < C) {
    s = 0.0;
    q = 0.0;
    for (int g = 0; g < RG; ++g) { s += red[0][g][tx]; q += red[1][g][tx]; }
    const double mean = s / count;
    double var = q / count - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = gamma[c] * invstd;
    coef[c] = (float)mean;
    coef[C + c] = invstd;
    coef[2 * C + c] = sc;
    coef[3 * C + c] = beta[c] - (float)mean * sc;
    if (rmean) {
      const double unb = count > 1.0 ? var * count / (count - 1.0) : var;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mean;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
    }
  }
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
}

// eval-mode coefficients from running stats
__global__ void bn_eval_coef_kernel(int C, const float* gamma, const float* beta, const float* rmean,
                                    const float* rvar, float eps, float* coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = 1.0f / sqrtf(rvar[c] + eps);
  const float sc = gamma[c] * invstd;
  coef[c] = rmean[c];
  coef[C + c] = invstd;
  coef[2 * C + c] = sc;
  coef[3 * C + c] = beta[c] - rmean[c] * sc;
}

RDP_DEV void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = __uint_as_float(w[k] << 16);
    f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}
RDP_DEV uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2bf(f[0], f[1]);
  v.y = pack2bf(f[2], f[3]);
  v.z = pack2bf(f[4], f[5]);
  v.w = pack2bf(f[6], f[7]);
  return v;
}

RDP_DEV void ld8(const float* p, float* f) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// a = relu(y*scale + shift), 8 channels per thread
// Elementwise kernels: each thread owns ONE 8-channel group for the whole launch (its BN
// coefficients stay in registers) and walks pixels with a grid stride, APX pixels in flight
// (16-B loads), so the loop carries no division and no coefficient reloads.
#define APX 4
__global__ __launch_bounds__(256) void bn_relu_apply_kernel(const u16* __restrict__ y, int ypitch,
                                                            u16* __restrict__ out, int opitch,
                                                            const float* __restrict__ coef, int M, int C, int relu,
                                                            int chunk) {
  const int CG = C >> 3, RPB = 256 / CG;  // C is a power of two in [8, 2048]
  const int g = threadIdx.x & (CG - 1), r = threadIdx.x / CG;
  const int c = g * 8;
  float ss[8], hh[8];
  ld8(coef + 2 * C + c, ss);
  ld8(coef + 3 * C + c, hh);
  // chunk > 0: block b walks pixels [b * chunk, (b + 1) * chunk) contiguously (RPB * APX per step)
  const int stride = chunk ? RPB : gridDim.x * RPB;
  const int pbeg = chunk ? blockIdx.x * chunk : blockIdx.x * RPB;
  const int pend = chunk ? min(M, pbeg + chunk) : M;
  for (int p0 = pbeg + r; p0 < pend; p0 += stride * APX) {
    uint4 v[APX];
#pragma unroll
    for (int u = 0; u < APX; ++u) {
      const int p = p0 + u * stride;
      if (p < pend) v[u] = *(const uint4*)(y + (size_t)p * ypitch + c);
    }
#pragma unroll
    for (int u = 0; u < APX; ++u) {
      const int p = p0 + u * stride;
      if (p < pend) {
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float z = fmaf(f[k], ss[k], hh[k]);
          f[k] = relu ? fmaxf(z, 0.f) : z;
        }
        *(uint4*)(out + (size_t)p * opitch + c) = pack8(f);
      }
    }
  }
}

// Backward reduce: partial[blk][0][c] = sum g, partial[blk][1][c] = sum g*xhat,
// g = da * (y*scale+shift > 0), xhat = (y-mean)*invstd.
__global__ __launch_bounds__(256) void bn_relu_bwd_reduce_kernel(const u16* __restrict__ da, int dapitch,
                                                                 const u16* __restrict__ y, int ypitch,
                                                                 const float* __restrict__ coef, int M, int C,
                                                                 int relu, float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float sred[];  // [rows][C][2]
  const int CG = C >> 3;
  const int rows = 256 / CG;  // pixel rows processed in parallel by the block
  const int g = threadIdx.x % CG, r = threadIdx.x / CG;
  const int c = g * 8;
  float mean[8], inv[8], ss[8], hh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mean[k] = coef[c + k];
    inv[k] = coef[C + c + k];
    ss[k] = coef[2 * C + c + k];
    hh[k] = coef[3 * C + c + k];
  }
  float sg[8], sgx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { sg[k] = 0.f; sgx[k] = 0.f; }
  if (r < rows) {
    for (long p = blockIdx.x * (long)rows + r; p < M; p += (long)gridDim.x * rows) {
      float fd[8], fy[8];
      unpack8(*(const uint4*)(da + (size_t)p * dapitch + c), fd);
      unpack8(*(const uint4*)(y + (size_t)p * ypitch + c), fy);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float gg = (!relu || fmaf(fy[k], ss[k], hh[k]) > 0.f) ? fd[k] : 0.f;
        sg[k] += gg;
        sgx[k] += gg * (fy[k] - mean[k]) * inv[k];
      }
    }
  }
  const int R = rows;
  if (r < R) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sred[(r * C + c + k) * 2] = sg[k];
      sred[(r * C + c + k) * 2 + 1] = sgx[k];
    }
  }
  __syncthreads();
  for (int cc = threadIdx.x; cc < C; cc += 256) {
    float a0 = 0.f, a1 = 0.f;
    for (int q = 0; q < R; ++q) { a0 += sred[(q * C + cc) * 2]; a1 += sred[(q * C + cc) * 2 + 1]; }
    partial[(size_t)blockIdx.x * 2 * C + cc] = a0;
    partial[(size_t)blockIdx.x * 2 * C + C + cc] = a1;
  }
}

// Backward finalize: dgamma, dbeta (written or accumulated into fp32 grads) and the apply
// coefficients coef2 = [A | B | Cc]: dy = A*g + B*y + Cc.
template <int CPB>
__global__ __launch_bounds__(64 * FIN_RG) void bn_bwd_finalize_kernel(const float* __restrict__ partial, int T, int C, double count,
                                       const float* __restrict__ gamma, const float* __restrict__ coef,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta,
                                       float* __restrict__ coef2) {
  constexpr int RG = 64 * FIN_RG / CPB;
  __shared__ double red[2][RG][CPB];
  const int tx = threadIdx.x % CPB, ty = threadIdx.x / CPB;
  const int c = blockIdx.x * CPB + tx;
  double s = 0.0, q = 0.0;
  if (c < C) fin_rows<RG>(partial, T, C, c, ty, s, q);
  red[0][ty][tx] = s;
  red[1][ty][tx] = q;
  __syncthreads();
  if (ty == 0 && c < C) {
    s = 0.0;
    q = 0.0;
    for (int g = 0; g < RG; ++g) { s += red[0][g][tx]; q += red[1][g][tx]; }
    if (dbeta) dbeta[c] = (float)s;
    if (dgamma) dgamma[c] = (float)q;
    const double mean = coef[c], inv = coef[C + c], gm = gamma[c];
    const double A = gm * inv;
    const double mg = s / count, mgx = q / count;
    coef2[c] = (float)A;
    coef2[C + c] = (float)(-A * inv * mgx);
    coef2[2 * C + c] = (float)(-A * mg + A * inv * mgx * mean);
  }
}

__global__ __launch_bounds__(256) void bn_relu_bwd_apply_kernel(const u16* __restrict__ da, int dapitch,
                                                                const u16* __restrict__ y, int ypitch,
                                                                const float* __restrict__ coef,
                                                                const float* __restrict__ coef2,
                                                                u16* __restrict__ dy, int dypitch, int M, int C,
                                                                int relu, int chunk) {
  const int CG = C >> 3, RPB = 256 / CG;
  const int g = threadIdx.x & (CG - 1), r = threadIdx.x / CG;
  const int c = g * 8;
  float ss[8], hh[8], A[8], B[8], K[8];
  ld8(coef + 2 * C + c, ss); ld8(coef + 3 * C + c, hh);
  ld8(coef2 + c, A); ld8(coef2 + C + c, B); ld8(coef2 + 2 * C + c, K);
  const int stride = chunk ? RPB : gridDim.x * RPB;  // (see bn_relu_apply_kernel)
  const int pbeg = chunk ? blockIdx.x * chunk : blockIdx.x * RPB;
  const int pend = chunk ? min(M, pbeg + chunk) : M;
  for (int p0 = pbeg + r; p0 < pend; p0 += stride * APX) {
    uint4 vd[APX], vy[APX];
#pragma unroll
    for (int u = 0; u < APX; ++u) {
      const int p = p0 + u * stride;
      if (p < pend) {
        vd[u] = *(const uint4*)(da + (size_t)p * dapitch + c);
        vy[u] = *(const uint4*)(y + (size_t)p * ypitch + c);
      }
    }
#pragma unroll
    for (int u = 0; u < APX; ++u) {
      const int p = p0 + u * stride;
      if (p < pend) {
        float fd[8], fy[8], o[8];
        unpack8(vd[u], fd);
        unpack8(vy[u], fy);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float gg = (!relu || fmaf(fy[k], ss[k], hh[k]) > 0.f) ? fd[k] : 0.f;
          o[k] = fmaf(A[k], gg, fmaf(B[k], fy[k], K[k]));
        }
        *(uint4*)(dy + (size_t)p * dypitch + c) = pack8(o);
      }
    }
  }
}

static bool pow2_channels(int C) { return C >= 8 && C <= 2048 && (C & (C - 1)) == 0; }

static int grid_px(long M, int C) {  // blocks for the pixel-walking elementwise kernels
  const long rpb = 256 / (C / 8);
  const long g = (M + rpb * APX - 1) / (rpb * APX);
  return (int)std::max<long>(1, std::min<long>(g, 2048));
}
// Contiguous per-block pixel chunks for the streaming BN apply passes: each block walks its own range
// (RPB * APX pixels per step) instead of a grid stride that keeps ~2,048 x APX far-apart streams open.
// Measured (scripts/pass_bench.py, bs 64): apply 256^2 x 64 256 -> 204 us (4.2 -> 5.3 TB/s), backward
// apply 383 -> 305 us, 128^2 x 128 182 -> 155 us; step 19.32 / 19.31 -> 19.22 / 19.21 ms (interleaved).
static int px_chunk(long M, int C, int grid) {
  const long step = (long)(256 / (C / 8)) * APX;
  return (int)(((M + grid - 1) / grid + step - 1) / step * step);
}

extern "C" {

int rdp_bn_finalize(const float* stats, int T, int C, long count, const float* gamma, const float* beta,
                    float* rmean, float* rvar, long long* nbt, float momentum, float eps, float* coef, float* ws,
                    hipStream_t s) {
  stats = shrink_rows(stats, T, 2 * C, ws, T, s);
  hipLaunchKernelGGL(bn_finalize_kernel<64>, dim3((C + 63) / 64), dim3(64 * FIN_RG), 0, s, stats, T, C, (double)count, gamma,
                     beta, rmean, rvar, nbt, momentum, eps, coef);
  return 0;
}

int rdp_rows_fold(const float* buf, int T, int K, double* out, hipStream_t s) {
  if (T < 1 || K < 1) return -1;
  hipLaunchKernelGGL(rows_fold_kernel, dim3((K + 63) / 64), dim3(1024), 0, s, buf, T, K, out);
  return 0;
}

int rdp_rows_hilo(const double* in, float* buf, int K, hipStream_t s) {
  if (K < 1) return -1;
  hipLaunchKernelGGL(rows_hilo_kernel, dim3((K + 255) / 256), dim3(256), 0, s, in, buf, K);
  return 0;
}

int rdp_bn_eval_coef(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar, float eps,
                     float* coef, hipStream_t s) {
  hipLaunchKernelGGL(bn_eval_coef_kernel, dim3((C + 63) / 64), dim3(64), 0, s, C, gamma, beta, rmean, rvar, eps, coef);
  return 0;
}

int rdp_bn_relu_apply(const void* y, int ypitch, void* out, int opitch, const float* coef, int M, int C, int relu,
                      hipStream_t s) {
  if (!pow2_channels(C) || ypitch % 8 || opitch % 8) return -1;
  const int grid = grid_px(M, C);
  hipLaunchKernelGGL(bn_relu_apply_kernel, dim3(grid), dim3(256), 0, s, (const u16*)y, ypitch, (u16*)out,
                     opitch, coef, M, C, relu, px_chunk(M, C, grid));
  return 0;
}

// returns the number of partial rows written (T for bn_bwd_finalize)
int rdp_bn_relu_bwd_reduce(const void* da, int dapitch, const void* y, int ypitch, const float* coef, int M, int C,
                           int relu, float* partial, int max_blocks, hipStream_t s) {
  if (C % 8 || C > 2048) return -1;
  const int rows = 256 / (C / 8);
  int blocks = (int)std::min<long>(max_blocks, ((long)M + rows * 8 - 1) / (rows * 8));
  if (blocks < 1) blocks = 1;
  const size_t lds = (size_t)rows * C * 2 * sizeof(float);
  hipLaunchKernelGGL(bn_relu_bwd_reduce_kernel, dim3(blocks), dim3(256), lds, s, (const u16*)da, dapitch,
                     (const u16*)y, ypitch, coef, M, C, relu, partial);
  return blocks;
}

int rdp_bn_bwd_finalize(const float* partial, int T, int C, long count, const float* gamma, const float* coef,
                        float* dgamma, float* dbeta, float* coef2, float* ws, hipStream_t s) {
  partial = shrink_rows(partial, T, 2 * C, ws, T, s);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<64>, dim3((C + 63) / 64), dim3(64 * FIN_RG), 0, s, partial, T, C, (double)count, gamma,
                     coef, dgamma, dbeta, coef2);
  return 0;
}

int rdp_bn_relu_bwd_apply(const void* da, int dapitch, const void* y, int ypitch, const float* coef,
                          const float* coef2, void* dy, int dypitch, int M, int C, int relu, hipStream_t s) {
  if (!pow2_channels(C) || dapitch % 8 || ypitch % 8 || dypitch % 8) return -1;
  const int grid = grid_px(M, C);
  hipLaunchKernelGGL(bn_relu_bwd_apply_kernel, dim3(grid), dim3(256), 0, s, (const u16*)da, dapitch,
                     (const u16*)y, ypitch, coef, coef2, (u16*)dy, dypitch, M, C, relu, px_chunk(M, C, grid));
  return 0;
}

}  // extern "C"

// Fused Adam over ONE flat fp32 master buffer + bf16 weight shadows for the conv kernels.
//
// Reference: torch.optim.Adam(model.parameters(), lr=1e-4) (/root/reference/scripts/train_segmenter.py:144,163),
// default betas (0.9, 0.999), eps 1e-8, no weight decay, bias correction. Math mirrors torch's:
//   m = lerp(m, g, 1-b1); v = b2*v + (1-b2)*g*g;
//   p -= (lr / (1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
// The step counter lives on the device (hipGraph-replayable); `gscale` folds the 1/world DDP
// average into the update. Each updated value is also written as bf16 into the flat shadow
// (identity layout = the forward conv weights, OHWI).
// wprep builds the derived bf16 layouts from the fp32 masters in one launch (segment table):
//   kind 0: dgrad weights  Wt[cin][8-tap][cout] = W[cout][tap][cin]   (flip + transpose)
//   kind 1: packed first layer  Wp[cout][16][8] (taps 0..8, channels 0..cin-1, zeros elsewhere)
#include "common.h"
#include <algorithm>
#include <stdlib.h>

// G = float (the flat fp32 gradient) or u16: bf16 gradients straight from the DDP bf16 all-reduce
// buffer (parallel/ddp.py comm_dtype), widened here instead of by a separate pass.
template <typename G>
__global__ void adam_kernel(float* __restrict__ p, const G* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, u16* __restrict__ shadow, long n, float lr, float b1, float b2,
                            float eps, float wd, float gscale, const int* __restrict__ step) {
  const int t = step[0] + 1;
  const float bc1 = 1.f - (float)pow((double)b1, (double)t);
  const float bc2 = 1.f - (float)pow((double)b2, (double)t);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  const long n4 = n >> 2;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pp = ((float4*)p)[i], gg, mm = ((float4*)m)[i], vv = ((float4*)v)[i];
    if constexpr (sizeof(G) == 4) {
      gg = ((const float4*)g)[i];
    } else {
      const uint2 gb = ((const uint2*)g)[i];
      gg = make_float4(__uint_as_float(gb.x << 16), __uint_as_float(gb.x & 0xffff0000u),
                       __uint_as_float(gb.y << 16), __uint_as_float(gb.y & 0xffff0000u));
    }
    float* pa = &pp.x; float* ga = &gg.x; float* ma = &mm.x; float* va = &vv.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gk = ga[k] * gscale;
      if (wd != 0.f) gk = fmaf(wd, pa[k], gk);
      ma[k] = ma[k] + (1.f - b1) * (gk - ma[k]);
      va[k] = va[k] * b2 + (1.f - b2) * gk * gk;
      const float den = sqrtf(va[k]) / bc2s + eps;
      pa[k] = pa[k] - step_size * ma[k] / den;
    }
    ((float4*)p)[i] = pp;
    ((float4*)m)[i] = mm;
    ((float4*)v)[i] = vv;
    if (shadow) {
      uint2 o;
      o.x = pack2bf(pp.x, pp.y);
      o.y = pack2bf(pp.z, pp.w);
      ((uint2*)shadow)[i] = o;
    }
  }
}

__global__ void step_inc_kernel(int* step) { step[0] += 1; }

__global__ void cast_bf16_kernel(const float* __restrict__ p, u16* __restrict__ out, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) out[i] = f2bf(p[i]);
}

struct WSeg {
  long src;  // element offset in the fp32 master
  long dst;  // element offset in the bf16 derived buffer
  int kind, cout, cin, taps;
};

// kind 0 is a per-tap 2-D transpose ([cout][cin] -> [cin][cout]); it goes through a 64x64 LDS tile
// so both the fp32 reads (along cin) and the bf16 writes (along cout) are coalesced. (The direct
// element-wise gather read the masters with a stride of taps*cin floats: ~130 us per step.)
// step != nullptr: also advance Adam's device step counter (the optimizer step just ran on the
// same stream, so every Adam block has read it) -- one launch fewer than a separate increment
__global__ __launch_bounds__(256) void wprep_kernel(const float* __restrict__ master, u16* __restrict__ out,
                                                    const WSeg* __restrict__ segs, int* __restrict__ step) {
  const WSeg sg = segs[blockIdx.y];
  const int tid = threadIdx.x;
  if (step && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) step[0] += 1;
  if (sg.kind == 0) {
    __shared__ u16 tile[64][66];
    const int tco = (sg.cout + 63) >> 6, tci = (sg.cin + 63) >> 6;
    const int ntiles = sg.taps * tco * tci;
    const int lc = tid & 63, lr = tid >> 6;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
      const int tap = t % sg.taps, r = t / sg.taps;
      const int co0 = (r % tco) << 6, ci0 = (r / tco) << 6;
      const int ci = ci0 + lc;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int co = co0 + lr + 4 * j;
        float v = 0.f;
        if (co < sg.cout && ci < sg.cin) v = master[sg.src + ((long)co * sg.taps + tap) * sg.cin + ci];
        tile[lr + 4 * j][lc] = f2bf(v);
      }
      __syncthreads();
      const int tp = sg.taps - 1 - tap, co = co0 + lc;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int ci2 = ci0 + lr + 4 * j;
        if (co < sg.cout && ci2 < sg.cin) out[sg.dst + ((long)ci2 * sg.taps + tp) * sg.cout + co] = tile[lc][lr + 4 * j];
      }
      __syncthreads();
    }
  } else {
    const long n = (long)sg.cout * 128;
    for (long i = blockIdx.x * (long)blockDim.x + tid; i < n; i += (long)gridDim.x * blockDim.x) {
      const int c = i % 8, tap = (i / 8) % 16, co = i / 128;
      float val = 0.f;
      if (tap < sg.taps && c < sg.cin) val = master[sg.src + ((long)co * sg.taps + tap) * sg.cin + c];
      out[sg.dst + i] = f2bf(val);
    }
  }
}

extern "C" {
// inc = 0: the caller advances the step counter later on this stream (rdp_wprep with step)
// g_bf16: g is bf16 (u16) instead of fp32
// max_blocks > 0 caps the grid (grid-stride loop): the overlapped update on the side stream leaves CUs to
// the next forward's first layers
int rdp_adam(float* p, const void* g, int g_bf16, float* m, float* v, void* shadow, long n, float lr, float b1,
             float b2, float eps, float wd, float gscale, int* step, int inc, int max_blocks, hipStream_t s) {
  if (n % 4) return -1;
  const long n4 = n / 4;
  int grid = (int)std::max<long>(1, std::min<long>((n4 + 255) / 256, 8192));
  if (max_blocks > 0 && grid > max_blocks) grid = max_blocks;
  if (g_bf16)
    hipLaunchKernelGGL(adam_kernel<u16>, dim3(grid), dim3(256), 0, s, p, (const u16*)g, m, v, (u16*)shadow, n, lr, b1,
                       b2, eps, wd, gscale, step);
  else
    hipLaunchKernelGGL(adam_kernel<float>, dim3(grid), dim3(256), 0, s, p, (const float*)g, m, v, (u16*)shadow, n, lr,
                       b1, b2, eps, wd, gscale, step);
  if (inc) hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, s, step);
  return 0;
}

int rdp_cast_bf16(const float* p, void* out, long n, hipStream_t s) {
  const int grid = (int)std::max<long>(1, std::min<long>((n + 255) / 256, 8192));
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid), dim3(256), 0, s, p, (u16*)out, n);
  return 0;
}

// segs: device array of nseg WSeg {long src, long dst, int kind, cout, cin, taps} (32 bytes each);
// blocks: blocks per segment (0: 1152, enough for the largest layer; the caller passes the table's own
// need -- e.g. 32 for the packed first layer alone -- so a small table is not a 1152-block launch)
int rdp_wprep(const float* master, void* out, const void* segs, int nseg, int* step, int blocks, hipStream_t s) {
  if (nseg <= 0) {
    if (step) hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, s, step);
    return 0;
  }
  // blocks per segment: the largest layer (512 x 1024 x 9) has 1152 64x64 tiles; at 128 blocks per
  // segment every block of it walked 9 tiles back to back (latency-bound: 68 us per step, a fixed
  // cost at every batch size). Blocks of smaller segments past their tile count exit at once.
  const int gx = blocks > 0 ? std::min(blocks, 1152) : 1152;
  hipLaunchKernelGGL(wprep_kernel, dim3(gx, nseg), dim3(256), 0, s, master, (u16*)out, (const WSeg*)segs, step);
  return 0;
}
int rdp_wseg_size() { return (int)sizeof(WSeg); }
}

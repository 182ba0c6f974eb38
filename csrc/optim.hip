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
  int tile0;  // first work tile of this segment in the table's flat tile range
  int pad;
};

// Work tiles of a segment: kind 0 = one 64 x 64 (cout x cin) block of one tap, kind 1 = 256 threads x 8
// packed elements. The table carries each segment's first tile (tile0), so the launch is ONE flat range
// of real tiles (grid-strided) instead of a [max tiles] x [segments] grid that was mostly early-exit
// blocks.
RDP_DEV int wseg_tiles(const WSeg& sg) {
  return sg.kind == 0 ? sg.taps * ((sg.cout + 63) >> 6) * ((sg.cin + 63) >> 6) : (sg.cout * 128 + 2047) >> 11;
}

// kind 0 is a per-tap 2-D transpose ([cout][cin] -> [cin][cout]) through a 64 x 64 bf16 LDS tile:
// fp32 masters read as 16-B vectors along cin (a 64-float row = one full 256-B line per 16 lanes),
// converted to bf16 and scattered transposed into LDS ([cin][cout]); the bf16 rows go out as 16-B
// vectors along cout (128 B per cin row). The first form moved 4-B loads / 2-B stores per element
// through a [cout][cin] tile (430 us of shared CU time per bs-64 step beside the forward, 67 us alone
// at bs 4: profiles/train_step_kernels.md). Segments with cin % 4, cout % 8 or unaligned offsets take the
// scalar path (the model's 64-element parameter alignment never does).
// step != nullptr: also advance Adam's device step counter (the optimizer step just ran on the
// same stream, so every Adam block has read it) -- one launch fewer than a separate increment
__global__ __launch_bounds__(256) void wprep_kernel(const float* __restrict__ master, u16* __restrict__ out,
                                                    const WSeg* __restrict__ segs, int nseg, int total,
                                                    int* __restrict__ step) {
  __shared__ __attribute__((aligned(16))) u16 tile[64][72];  // [cin][cout], 144-B rows (16-B aligned)
  const int tid = threadIdx.x;
  if (step && blockIdx.x == 0 && tid == 0) step[0] += 1;
  for (int t = blockIdx.x; t < total; t += gridDim.x) {
    int si = 0;  // segment of tile t (tables hold a few dozen segments: linear scan, uniform)
    while (si + 1 < nseg && segs[si + 1].tile0 <= t) ++si;
    const WSeg sg = segs[si];
    const int lt = t - sg.tile0;
    if (sg.kind == 0) {
      const int tco = (sg.cout + 63) >> 6;
      const int tap = lt % sg.taps, r = lt / sg.taps;
      const int co0 = (r % tco) << 6, ci0 = (r / tco) << 6;
      const int tp = sg.taps - 1 - tap;
      if ((sg.cin & 3) == 0 && (sg.cout & 7) == 0 && (sg.src & 3) == 0 && (sg.dst & 7) == 0) {
        // read: thread -> (cout row co0 + (tid >> 4) + 16 j, cin quad 4 (tid & 15))
        const int cq = 4 * (tid & 15);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int rco = (tid >> 4) + 16 * j, co = co0 + rco, ci = ci0 + cq;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (co < sg.cout && ci < sg.cin)
            v = *(const float4*)(master + sg.src + ((long)co * sg.taps + tap) * sg.cin + ci);
          tile[cq + 0][rco] = f2bf(v.x);
          tile[cq + 1][rco] = f2bf(v.y);
          tile[cq + 2][rco] = f2bf(v.z);
          tile[cq + 3][rco] = f2bf(v.w);
        }
        __syncthreads();
        // write: thread -> (cin row ci0 + (tid >> 3) + 32 j, 8 couts 8 (tid & 7))
        const int c8 = 8 * (tid & 7);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int rci = (tid >> 3) + 32 * j, ci2 = ci0 + rci, co = co0 + c8;
          if (ci2 < sg.cin && co < sg.cout)
            *(uint4*)(out + sg.dst + ((long)ci2 * sg.taps + tp) * sg.cout + co) = *(const uint4*)&tile[rci][c8];
        }
        __syncthreads();
      } else {
        const int lc = tid & 63, lr = tid >> 6;
        for (int j = 0; j < 16; ++j) {
          const int co = co0 + lr + 4 * j, ci = ci0 + lc;
          float v = 0.f;
          if (co < sg.cout && ci < sg.cin) v = master[sg.src + ((long)co * sg.taps + tap) * sg.cin + ci];
          tile[lc][lr + 4 * j] = f2bf(v);
        }
        __syncthreads();
        for (int j = 0; j < 16; ++j) {
          const int ci2 = ci0 + lr + 4 * j, co = co0 + lc;
          if (co < sg.cout && ci2 < sg.cin) out[sg.dst + ((long)ci2 * sg.taps + tp) * sg.cout + co] = tile[lr + 4 * j][lc];
        }
        __syncthreads();
      }
    } else {  // packed first layer: 8 consecutive elements (one tap's channel slots) per thread
      const long e0 = ((long)lt * 256 + tid) * 8, n = (long)sg.cout * 128;
      if (e0 < n) {
        const int tap = (int)((e0 >> 3) & 15), co = (int)(e0 >> 7);
        float f[8];
#pragma unroll
        for (int c = 0; c < 8; ++c)
          f[c] = (tap < sg.taps && c < sg.cin) ? master[sg.src + ((long)co * sg.taps + tap) * sg.cin + c] : 0.f;
        if ((sg.dst & 7) == 0)
          *(uint4*)(out + sg.dst + e0) =
              make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
        else
          for (int c = 0; c < 8; ++c) out[sg.dst + e0 + c] = f2bf(f[c]);
      }
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

// segs: device array of nseg WSeg {long src, long dst, int kind, cout, cin, taps, tile0, pad} (40 bytes
// each; tile0 = the running sum of wseg_tiles over the earlier segments); tiles = the table's total tile
// count (the caller's sum), blocks = grid cap (0: one block per tile, at most 4096)
int rdp_wprep(const float* master, void* out, const void* segs, int nseg, int* step, int tiles, int blocks,
              hipStream_t s) {
  if (nseg <= 0 || tiles <= 0) {
    if (step) hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, s, step);
    return 0;
  }
  const int gx = std::max(1, std::min(tiles, blocks > 0 ? blocks : 4096));
  hipLaunchKernelGGL(wprep_kernel, dim3(gx), dim3(256), 0, s, master, (u16*)out, (const WSeg*)segs, nseg, tiles, step);
  return 0;
}
int rdp_wseg_size() { return (int)sizeof(WSeg); }
}

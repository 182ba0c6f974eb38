// First U-Net layer: 3x3 conv (pad 1) of the 3-channel input to 64 output channels, NHWC bf16,
// MFMA 16x16x32, with the training BN-statistics or eval BN-fold(+ReLU) epilogue of conv_igemm.hip.
//
// Reference op: inc.double_conv.0 = nn.Conv2d(3, 64, 3, padding=1, bias=False)
// (/root/reference/pkg/segmentation_model.py:31) on the 256x256 RGB batch.
//
// The implicit-GEMM kernel runs this layer in its "packed" mode (8 taps x 8 channels per 64-wide K
// step, 2 K steps per 256-pixel tile): 66 TF/s at bs 64, 221 us for a layer whose floor is the
// 537 MB bf16 output write (~95 us at 5.6 TB/s) -- a 2-step K loop cannot hide the tile prologue,
// LDS-DMA round trips and epilogue. Here there is no LDS at all:
//   * K is re-packed as 16 taps x 4 channels (input channel 3 is the stored zero pad): one K step of
//     an MFMA is 8 taps, so the layer is 2 MFMAs per (16 couts x 16 pixels), tap 8 alone in the 2nd;
//   * a lane's A fragment (8 k = 2 taps x 4 channels of one pixel) is two 8-byte buffer loads of
//     the input pixel at the tap offset (zero padding from out-of-range offsets, L1/L2-resident:
//     the 3-channel input is 1/8 of the output bytes);
//   * the 64 x 64 packed weight fragments live in 32 VGPRs, loaded once per wave;
//   * a wave owns 64 consecutive pixels x 64 couts per step (4 x 4 accumulators) and walks the
//     pixel segments grid-stride; BN partial sums stay in registers until the wave's last segment,
//     then the block's 4 wave rows are summed through LDS into ONE stats row per block.
#include "common.h"
#include <algorithm>
#include <stdlib.h>

struct FirstArgs {
  const u16* x;  // [M][pitch], channels 0..3 read (3..7 are the zero pad of the 3-channel input)
  uint32_t xbytes;
  int pitch;
  const u16* w;  // packed [64][16 taps][8 ch] (conv_igemm "packed" layout), taps >= 9 / ch >= 3 zero
  uint32_t wbytes;
  u16* y;
  uint32_t ybytes;
  int ypitch;
  float* stats;  // [gridDim.x][2][64] partial (sum, sumsq) or nullptr
  const float* escale;  // eval BN fold: y = relu?(acc * escale + eshift)
  const float* eshift;
  int erelu;
  int H, W, M, nseg;
  uint32_t fhw_m, fhw_s, fw_m, fw_s;
};

RDP_DEV int ftap_dr(int tap) { return ((tap * 11) >> 5) - 1; }
RDP_DEV int ftap_ds(int tap) { return tap - 3 * ((tap * 11) >> 5) - 1; }

__global__ __launch_bounds__(256) void conv_first_kernel(const FirstArgs a) {
  __shared__ float red[4][2][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4;   // k group: taps 2g, 2g+1 of K step 0; tap 8 (g = 0) of K step 1
  const int pr = lane & 15;  // pixel (B) / cout (A) row within a 16-fragment
  const auto rx = make_rsrc(a.x, a.xbytes);
  const auto rw = make_rsrc(a.w, a.wbytes);
  const auto ry = make_rsrc(a.y, a.ybytes);

  // weight fragments: [j][K step], lane = (cout 16j + pr, taps of k group g), 4 channels per tap
  bf16x8 wf[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int t0 = 8 * s + 2 * g;
      const uint32_t base = (uint32_t)((16 * j + pr) * 128) * 2u;
      const uint2 lo = bload8(rw, base + (uint32_t)(t0 * 8) * 2u);
      const uint2 hi = bload8(rw, base + (uint32_t)((t0 + 1) * 8) * 2u);
      wf[j][s] = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
    }

  float s1[4][4], s2[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }

  const int gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;
  const int gq = lane >> 4;
  const int coff = 16 * (gq & 1) + 8 * (gq >> 1);
  // pixel fragments: [i][K step] for pixels seg*64 + 16i + pr.
  // Measured (scripts/first_layer_bench.py, bs 64, ablation builds): 221 us, 111 us without the output
  // stores, 111 us without the input gathers, 101 us with neither -- the 16 gather loads (8 B per
  // lane, 64 addresses) and 8 stores per segment share the vector-memory path and do not overlap;
  // issuing segment k+1's loads ahead of segment k's stores changed nothing at bs 64 and was slower at
  // bs 4 (14.7 -> 19.7 us), so the loop stays simple. At bs 64 this kernel ties the packed implicit
  // GEMM (~220 us; 3.1 TB/s of output incl. the gathers); at bs 4 / N = 1 it is 16 % / 15 % faster
  // (14.7 vs 17.5 us, 7.2 vs 8.6 us). The next step would be LDS-DMA row staging of the input (4 full-
  // line DMA instructions per segment instead of 16 gathers).
  auto load_px = [&](int seg, bf16x8 (&pf)[4][2]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = seg * 64 + 16 * i + pr;
      const bool valid = m < a.M;
      const uint32_t mm = valid ? (uint32_t)m : 0u;
      const uint32_t hw = mm - ((__umulhi(mm, a.fhw_m) + mm) >> a.fhw_s) * (uint32_t)(a.H * a.W);
      const int h = (int)((__umulhi(hw, a.fw_m) + hw) >> a.fw_s);
      const int w = (int)hw - h * a.W;
      uint2 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // taps 2g, 2g + 1 (step 0), 8 + 2g, 9 + 2g (step 1)
        const int tap = (q >> 1) * 8 + 2 * g + (q & 1);
        const int dr = ftap_dr(tap), ds = ftap_ds(tap);
        const bool ok = valid && tap < 9 && inb(h + dr, a.H) && inb(w + ds, a.W);
        const uint32_t off = ok ? (uint32_t)((m + dr * a.W + ds) * a.pitch) * 2u : RDP_OOB;
        v[q] = bload8(rx, off);
      }
      pf[i][0] = __builtin_bit_cast(bf16x8, make_uint4(v[0].x, v[0].y, v[1].x, v[1].y));
      pf[i][1] = __builtin_bit_cast(bf16x8, make_uint4(v[2].x, v[2].y, v[3].x, v[3].y));
    }
  };
  for (int seg = gw; seg < a.nseg; seg += nw) {
    bf16x8 pf[4][2];
    load_px(seg, pf);
    f32x4 acc[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][0], pf[i][0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][1], pf[i][1], acc[j][i], 0, 0, 0);
      }
    // epilogue (as conv_igemm_kernel): acc[j][i][r] = out[m = seg*64 + 16i + pr][n = 16j + 4 gq + r];
    // permlane16_swap of cout-fragment pairs gives every lane 8 consecutive couts = one 16-B store
#pragma unroll
    for (int jp = 0; jp < 4; jp += 2) {
      const int n = jp * 16 + coff;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = seg * 64 + 16 * i + pr;
        uint2 v[2];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int j = jp + hh;
          f32x4 o = acc[j][i];
          if (a.escale) {
            const int nc = jp * 16 + hh * 16 + 4 * gq;
            const float4 sc = *(const float4*)(a.escale + nc), sh = *(const float4*)(a.eshift + nc);
            o[0] = fmaf(o[0], sc.x, sh.x); o[1] = fmaf(o[1], sc.y, sh.y);
            o[2] = fmaf(o[2], sc.z, sh.z); o[3] = fmaf(o[3], sc.w, sh.w);
            if (a.erelu) {
              o[0] = fmaxf(o[0], 0.f); o[1] = fmaxf(o[1], 0.f); o[2] = fmaxf(o[2], 0.f); o[3] = fmaxf(o[3], 0.f);
            }
          }
          v[hh].x = pack2bf(o[0], o[1]);
          v[hh].y = pack2bf(o[2], o[3]);
          if (a.stats) {  // rows past M hold zeros (all taps read zeros): no contribution
            const float q0 = __uint_as_float(v[hh].x << 16), q1 = __uint_as_float(v[hh].x & 0xffff0000u);
            const float q2 = __uint_as_float(v[hh].y << 16), q3 = __uint_as_float(v[hh].y & 0xffff0000u);
            s1[j][0] += q0; s2[j][0] += q0 * q0;
            s1[j][1] += q1; s2[j][1] += q1 * q1;
            s1[j][2] += q2; s2[j][2] += q2 * q2;
            s1[j][3] += q3; s2[j][3] += q3 * q3;
          }
        }
        const auto rxs = __builtin_amdgcn_permlane16_swap(v[0].x, v[1].x, false, false);
        const auto rys = __builtin_amdgcn_permlane16_swap(v[0].y, v[1].y, false, false);
        const uint32_t off = m < a.M ? (uint32_t)(m * a.ypitch + n) * 2u : RDP_OOB;
        bstore16(ry, off, make_uint4(rxs[0], rys[0], rxs[1], rys[1]));
      }
    }
  }
  if (!a.stats) return;
  // one stats row per block: wave rows reduced over their 16 pixel lanes, then summed through LDS
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s1[j][r] = row16_sum(s1[j][r]);
      s2[j][r] = row16_sum(s2[j][r]);
    }
  if (pr == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 16 * j + 4 * gq;
      *(float4*)&red[wave][0][c] = make_float4(s1[j][0], s1[j][1], s1[j][2], s1[j][3]);
      *(float4*)&red[wave][1][c] = make_float4(s2[j][0], s2[j][1], s2[j][2], s2[j][3]);
    }
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int half = threadIdx.x >> 6, c = threadIdx.x & 63;
    const float t = (red[0][half][c] + red[1][half][c]) + (red[2][half][c] + red[3][half][c]);
    a.stats[(size_t)blockIdx.x * 128 + threadIdx.x] = t;
  }
}

// Returns the number of stats rows written (training) / 0, or -1 if the shape is not this kernel's
// (3-channel input stored with pitch >= 4, 64 couts, packed [64][128] weights).
extern "C" int rdp_conv_first(const void* x, long xbytes, int pitch, const void* w, long wbytes, void* y, long ybytes,
                              int ypitch, float* stats, int N, int H, int W, const float* escale, const float* eshift,
                              int erelu, hipStream_t s) {
  if (pitch < 4 || wbytes < 64l * 128 * 2 || ypitch < 64 || ypitch % 8) return -1;
  if (xbytes >= (1l << 31) || ybytes >= (1l << 31)) return -1;
  FirstArgs a;
  a.x = (const u16*)x; a.xbytes = (uint32_t)xbytes; a.pitch = pitch;
  a.w = (const u16*)w; a.wbytes = (uint32_t)wbytes;
  a.y = (u16*)y; a.ybytes = (uint32_t)ybytes; a.ypitch = ypitch;
  a.stats = stats; a.escale = escale; a.eshift = eshift; a.erelu = erelu;
  a.H = H; a.W = W; a.M = N * H * W;
  a.nseg = (a.M + 63) / 64;
  const FastDiv fhw = make_fastdiv((uint32_t)(H * W)), fw = make_fastdiv((uint32_t)W);
  a.fhw_m = fhw.m; a.fhw_s = fhw.s; a.fw_m = fw.m; a.fw_s = fw.s;
  // grid <= nseg / 4 keeps the stats rows within conv_stats_rows() (>= M / 32 rows)
  const int grid = std::max(1, std::min((a.nseg + 3) / 4, 512));
  hipLaunchKernelGGL(conv_first_kernel, dim3(grid), dim3(256), 0, s, a);
  return stats ? grid : 0;
}

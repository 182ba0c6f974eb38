// Row-band convolution for small eval feature maps (serving at N = 1: the 128^2 .. 16^2 levels),
// NHWC bf16, 3x3, BN folded into the epilogue + ReLU, optional fused MaxPool2d(2).
//
// Replaces, at these sizes, the implicit GEMM + split-K slab + reduce launch pair
// (csrc/conv_igemm.hip) for the eval U-Net the reference serves
// (/root/reference/services/vision_analysis/server.py:121-125 -> pkg/segmentation_model.py:31,34).
//
// Why a different structure: at N = 1 a deep conv has M = 256 .. 4096 pixels and K = 9 x 256 .. 9 x 1024.
// The LDS-staged GEMM tile needs split-K to fill 256 CUs, then pays a per-K-step block barrier on a
// two-deep DMA pipeline (~0.75 us per step at 1 block / CU), an fp32 slab round trip and a second
// launch. Here a block owns R image rows x 32 output channels with the WHOLE K, split over its 8 waves
// (wave w: the w-th eighth of the tap-major k-steps, 32 channels of one tap each). Both MFMA operands are
// read straight from global memory into registers -- a 16x16x32 bf16 fragment row is 8 consecutive
// channels, i.e. 16 contiguous bytes of NHWC activations or OHWI weights -- so a wave issues its loads
// G k-steps ahead with no barrier and no LDS until the end, where the 8 partial tiles are summed in LDS
// (fixed wave order: deterministic) and the epilogue (scale, shift, ReLU, bf16, optional 2x2 max) writes
// the rows. No slab, no second launch.
//
// Block -> tile: consecutive logical ids (one XCD after xcd_remap) are consecutive row bands of ONE
// 32-channel output slice, so that slice's weights (32 x 9 Cin bf16) are fetched into that XCD's L2
// once and re-read there by every band.
//
// Three forms live here:
//   * conv_rowband_kernel: the direct form above (OHWI or fragment-major weights);
//   * conv_rowband_x_kernel: fragment-major weights + each wave's 32-channel input chunk staged once per
//     tile in LDS for all 9 taps (the serving default wherever the input has 128 or 256k channels);
//   * conv_rowband_chain_kernel: the persistent multi-layer experiment (measured slower, kept tested).
// The eval dispatch is rdp_conv_rowband_frag_auto (bindings conv_fwd with the executor's fragment-major
// weights); rdp_conv_rowband_bytes is the OHWI form's traffic model used by rdp_conv_igemm.
#include "common.h"
#include <algorithm>
#include <stdlib.h>

struct RowbandArgs {
  const u16* x1;
  const u16* x2;
  uint32_t xbytes1, xbytes2;
  int C1, C2, pitch1, pitch2;
  const u16* w;
  uint32_t wbytes;
  int ldw;
  u16* y;
  uint32_t ybytes;
  int ypitch;
  u16* pool;  // MaxPool2d(2) of y, [N][H/2][W/2] (R == 2), or nullptr
  uint32_t pbytes;
  int ppitch;
  const float* escale;
  const float* eshift;
  int erelu;
  int N, H, W, Cout;
  int wshift;  // log2(W)
  int R;       // image rows per block
  int bands;   // H / R
  int cshift;  // log2(Cin / 32): k-step -> tap
  int T;       // k-steps = 9 * Cin / 32
  int wfrag;   // 1: w is fragment-major (models/unet.py rowband_frag_weights): 16 couts x 1 k-step = 1 KiB
  int segs;    // activation-staged variant: row segments of WB pixels per image row
};

// tap (0..8) -> (dr, ds) without division
RDP_DEV int rb_dr(int tap) { return ((tap * 11) >> 5) - 1; }
RDP_DEV int rb_ds(int tap) { return tap - 3 * ((tap * 11) >> 5) - 1; }

template <int NF, int NPG>
struct RbFrag {
  bf16x8 A[NF];   // weights: cout row (lane & 15) of fragment f, channels 8 (lane >> 4) .. +7
  bf16x8 B[NPG];  // pixels: pixel (lane & 15) of group g, channels 8 (lane >> 4) .. +7
};

template <int NF, int NPG>
struct RbSmem {
  f32x4 red[8][NF * NPG][64];   // the 8 waves' partial tiles
  uint2 ytile[NPG * 16][NF * 4];  // bf16 output tile for the fused pool
};

// One tile (row band x 32-channel slice, logical id lid) of layer a; the caller's LDS. WT: write-through
// (sc1) output stores, for an in-launch consumer on another XCD (the chain)
template <int NF, int NPG, int G, bool WT = false>
RDP_DEV void rowband_tile(const RowbandArgs& a, uint32_t lid, RbSmem<NF, NPG>& sm) {
  constexpr int NWV = 8, NC = NF * 16;
  auto& red = sm.red;
  auto& ytile = sm.ytile;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nb = a.N * a.bands;
  const int ct = (int)lid / nb, band = (int)lid - ct * nb;
  const int img = band / a.bands, h0 = (band - img * a.bands) * a.R;
  const int cout0 = ct * NC;

  const auto rx1 = make_rsrc(a.x1, a.xbytes1);
  const auto rx2 = make_rsrc(a.x2 ? a.x2 : a.x1, a.x2 ? a.xbytes2 : 0u);
  const auto rw = make_rsrc(a.w, a.wbytes);

  const int lr = lane & 15, lk = 8 * (lane >> 4);
  uint32_t wrow[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f)
    wrow[f] = a.wfrag ? (uint32_t)((cout0 / 16 + f) * a.T) * 1024u + (uint32_t)lane * 16u
                      : (uint32_t)((cout0 + 16 * f + lr) * a.ldw + lk) * 2u;
  const uint32_t wstep = a.wfrag ? 1024u : 64u;  // bytes per k-step
  int ph[NPG], pw[NPG];
#pragma unroll
  for (int g = 0; g < NPG; ++g) {
    const int p = 16 * g + lr;
    ph[g] = h0 + (p >> a.wshift);
    pw[g] = p & (a.W - 1);
  }
  const int ks0 = wave * a.T / NWV, ks1 = (wave + 1) * a.T / NWV;

  typedef RbFrag<NF, NPG> Frag;
  auto load = [&](int ks, Frag& fr) {
    const bool live = ks < ks1;
    const int tap = ks >> a.cshift;
    const int cbase = (ks - (tap << a.cshift)) << 5;  // first channel of the k-step (wave-uniform)
    const int dr = rb_dr(tap), ds = rb_ds(tap);
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const uint32_t off = live ? wrow[f] + (uint32_t)ks * wstep : RDP_OOB;
      fr.A[f] = __builtin_bit_cast(bf16x8, bload16(rw, off));
    }
    const bool s2 = cbase >= a.C1;
    const int pitch = s2 ? a.pitch2 : a.pitch1;
    const int ch = (s2 ? cbase - a.C1 : cbase) + lk;
#pragma unroll
    for (int g = 0; g < NPG; ++g) {
      const int hh = ph[g] + dr, ww = pw[g] + ds;
      const bool ok = live & inb(hh, a.H) & inb(ww, a.W);
      const uint32_t off = ok ? (uint32_t)((((img * a.H + hh) << a.wshift) + ww) * pitch + ch) * 2u : RDP_OOB;
      fr.B[g] = __builtin_bit_cast(bf16x8, bload16(s2 ? rx2 : rx1, off));
    }
  };

  f32x4 acc[NF][NPG];
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int g = 0; g < NPG; ++g) acc[f][g] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto comp = [&](const Frag* fr) {
#pragma unroll
    for (int i = 0; i < G; ++i)
#pragma unroll
      for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int g = 0; g < NPG; ++g)
          acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[i].A[f], fr[i].B[g], acc[f][g], 0, 0, 0);
  };
  auto load_g = [&](int k, Frag* fr) {
#pragma unroll
    for (int i = 0; i < G; ++i) load(k + i, fr[i]);
  };

  // two register buffers of G k-steps: the next group's loads are in flight while this one computes
  Frag fa[G], fb[G];
  int k = ks0;
  if (k < ks1) {
    load_g(k, fa);
    while (true) {
      if (k + G < ks1) load_g(k + G, fb);
      comp(fa);
      k += G;
      if (k >= ks1) break;
      if (k + G < ks1) load_g(k + G, fa);
      comp(fb);
      k += G;
      if (k >= ks1) break;
    }
  }

#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int g = 0; g < NPG; ++g) red[wave][f * NPG + g][lane] = acc[f][g];
  __syncthreads();

  const auto ry = make_rsrc(a.y, a.ybytes);
  for (int u = threadIdx.x; u < NF * NPG * 64; u += NWV * 64) {
    const int q = u >> 6, l = u & 63;
    f32x4 v = red[0][q][l];
#pragma unroll
    for (int w = 1; w < NWV; ++w) v += red[w][q][l];
    const int f = q / NPG, g = q - f * NPG;
    const int cl = 16 * f + 4 * (l >> 4);  // first of this lane's 4 output channels (within the tile)
    const int c = cout0 + cl;
    const float4 sc = *(const float4*)(a.escale + c), sh = *(const float4*)(a.eshift + c);
    float o[4] = {fmaf(v[0], sc.x, sh.x), fmaf(v[1], sc.y, sh.y), fmaf(v[2], sc.z, sh.z), fmaf(v[3], sc.w, sh.w)};
    if (a.erelu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = fmaxf(o[r], 0.f);
    }
    const uint2 pk = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
    const int p = 16 * g + (l & 15);
    const int m = ((img * a.H + h0 + (p >> a.wshift)) << a.wshift) + (p & (a.W - 1));
    __builtin_amdgcn_raw_buffer_store_b64(*reinterpret_cast<const __attribute__((ext_vector_type(2))) uint32_t*>(&pk), ry,
                                          (uint32_t)(m * a.ypitch + c) * 2u, 0, WT ? 16 : 0);
    if (a.pool) ytile[p][cl >> 2] = pk;
  }
  if (!a.pool) return;  // block-uniform
  __syncthreads();
  // 2 x 2 max of the block's two rows: W / 2 pooled pixels x NC / 4 channel quads
  const auto rp = make_rsrc(a.pool, a.pbytes);
  const int Wo = a.W >> 1;
  for (int u = threadIdx.x; u < Wo * (NC / 4); u += NWV * 64) {
    const int wo = u / (NC / 4), cq = u - wo * (NC / 4);
    const int p00 = 2 * wo, p10 = a.W + 2 * wo;
    const uint2 q[4] = {ytile[p00][cq], ytile[p00 + 1][cq], ytile[p10][cq], ytile[p10 + 1][cq]};
    float mx[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t wd = e < 2 ? q[0].x : q[0].y;
      mx[e] = __uint_as_float((e & 1) ? (wd & 0xffff0000u) : (wd << 16));
    }
#pragma unroll
    for (int t = 1; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t wd = e < 2 ? q[t].x : q[t].y;
        mx[e] = fmaxf(mx[e], __uint_as_float((e & 1) ? (wd & 0xffff0000u) : (wd << 16)));
      }
    const int mo = (img * (a.H >> 1) + (h0 >> 1)) * Wo + wo;
    bstore8(rp, (uint32_t)(mo * a.ppitch + cout0 + 4 * cq) * 2u, make_uint2(pack2bf(mx[0], mx[1]), pack2bf(mx[2], mx[3])));
  }
}

// Two blocks per CU (<= 128 VGPRs: G k-steps of operands per register buffer). (16-wave blocks, K split
// twice as finely, and 8-wave blocks at one per CU with deeper register buffers measured the same:
// scripts/rowband_bench.py -- the kernel is bound by the L2 -> CU operand bytes, not by load latency.)
template <int NF, int NPG, int G>
__global__ __launch_bounds__(512, 4) void conv_rowband_kernel(const RowbandArgs a) {
  __shared__ RbSmem<NF, NPG> sm;
  rowband_tile<NF, NPG, G>(a, xcd_remap(blockIdx.x, gridDim.x), sm);
}

// ---------------------------------------------------------------------------------------------
// Activation-staged variant (fragment-major weights only): the direct kernel reads every activation once
// per tap (9x per 32-channel output slice) as 16 half cache lines per load. Here wave w owns the 32-channel
// input chunks [w CC / 8, (w + 1) CC / 8) of all 9 taps; per chunk it stages the (R + 2) x (WB + 2) input
// pixels x 32 channels of its tile ONCE into its own LDS region (zero halo from out-of-range offsets), and
// the 9 taps read their shifted B fragments from there (16-B chunks XOR-swizzled by region column: the 16
// pixels of a fragment hit 16 distinct 4-bank groups). Only this wave writes and reads its region, so no
// block barrier is needed until the partial-tile exchange, which reuses the regions' LDS. A block owns
// R image rows x WB (<= 32) pixels of one row segment x 32 output channels.
template <int NPG, int R>
__global__ __launch_bounds__(512, 2) void conv_rowband_x_kernel(const RowbandArgs a) {
  constexpr int NF = 2, NWV = 8, NC = 32, PB = NPG * 16, WB = PB / R;
  constexpr int RW = WB + 2, RR = R + 2;
  constexpr int RBYTES = RR * RW * 64;
  constexpr int NIT = RR * RW * 4;            // 16-B staging items per region
  constexpr int NLD = (NIT + 63) / 64;        // per lane
  constexpr int REDB = NWV * NF * NPG * 64 * 16;
  constexpr int SMEM = NWV * RBYTES > REDB ? NWV * RBYTES : REDB;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  __shared__ uint2 ytile[PB][NC / 4];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lid = xcd_remap(blockIdx.x, gridDim.x);
  const int nb = a.N * a.bands * a.segs;  // tiles of one 32-channel output slice (consecutive: one XCD)
  const int ct = (int)lid / nb;
  int rem = (int)lid - ct * nb;
  const int seg = rem % a.segs;
  rem /= a.segs;
  const int band = rem % a.bands, img = rem / a.bands;
  const int h0 = band * R, w0 = seg * WB, cout0 = ct * NC;

  const auto rx1 = make_rsrc(a.x1, a.xbytes1);
  const auto rx2 = make_rsrc(a.x2 ? a.x2 : a.x1, a.x2 ? a.xbytes2 : 0u);
  const auto rw = make_rsrc(a.w, a.wbytes);
  char* const reg = smem + wave * RBYTES;
  typedef __attribute__((address_space(3))) void lds_t;

  // staging items of this lane: region pixel q = i >> 2 (row q / RW, column q % RW), 16-B part i & 3
  int spix[NLD], sdst[NLD];
#pragma unroll
  for (int t = 0; t < NLD; ++t) {
    const int i = lane + 64 * t, q = i >> 2, j = i & 3;
    const int rr = q / RW, cc = q - rr * RW;
    const int hh = h0 - 1 + rr, ww = w0 - 1 + cc;
    const bool ok = i < NIT && inb(hh, a.H) && inb(ww, a.W);
    spix[t] = ok ? ((img * a.H + hh) << a.wshift) + ww : -1;
    sdst[t] = i < NIT ? q * 64 + 16 * (j ^ ((cc >> 2) & 3)) : -1;
  }
  uint4 xr[NLD];
  auto load_x = [&](int chunk) {
    const int cb = chunk * 32;
    const bool s2 = cb >= a.C1;  // wave-uniform
    const int pitch = s2 ? a.pitch2 : a.pitch1;
    const int ch = s2 ? cb - a.C1 : cb;
#pragma unroll
    for (int t = 0; t < NLD; ++t) {
      const int j = (lane + 64 * t) & 3;
      const uint32_t off = spix[t] >= 0 ? (uint32_t)(spix[t] * pitch + ch + 8 * j) * 2u : RDP_OOB;
      xr[t] = bload16(s2 ? rx2 : rx1, off);
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int t = 0; t < NLD; ++t)
      if (sdst[t] >= 0) *(uint4*)(reg + sdst[t]) = xr[t];
  };
  // B fragment geometry: block pixel p = 16 g + (lane & 15) -> tile row p / WB, column p % WB
  int brow[NPG], bcol[NPG];
#pragma unroll
  for (int g = 0; g < NPG; ++g) {
    const int p = 16 * g + (lane & 15);
    brow[g] = p / WB;
    bcol[g] = p - brow[g] * WB;
  }
  const int gq = lane >> 4;
  const int CC = a.T / 9;
  uint32_t wbase[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) wbase[f] = (uint32_t)((cout0 / 16 + f) * a.T) * 1024u + (uint32_t)lane * 16u;

  f32x4 acc[NF][NPG];
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int g = 0; g < NPG; ++g) acc[f][g] = f32x4{0.f, 0.f, 0.f, 0.f};

  // K split over the waves: >= 8 chunks -> whole chunks (all 9 taps) per wave; 2 or 4 chunks (64 / 128 input
  // channels) -> 8 / CC waves per chunk, each staging it and taking a range of its taps
  int c0, c1, t0 = 0, t1 = 9;
  if (CC >= NWV) {
    c0 = wave * CC / NWV;
    c1 = (wave + 1) * CC / NWV;
  } else {
    const int G = NWV / CC, part = wave % G;
    c0 = wave / G;
    c1 = c0 + 1;
    t0 = part * 9 / G;
    t1 = (part + 1) * 9 / G;
  }
  if (c0 < c1) {
    load_x(c0);
    store_x();
  }
  for (int chunk = c0; chunk < c1; ++chunk) {
    if (chunk + 1 < c1) load_x(chunk + 1);  // lands under this chunk's taps
    bf16x8 wa[2][3][NF];
    auto load_w = [&](int tg, bf16x8 (&dst)[3][NF]) {
#pragma unroll
      for (int tt = 0; tt < 3; ++tt) {
        const int tap = 3 * tg + tt;
        if (tap < t0 || tap >= t1) continue;  // wave-uniform
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          const int ks = tap * CC + chunk;  // tap-major k-step of the fragment-major layout
          dst[tt][f] = __builtin_bit_cast(bf16x8, bload16(rw, wbase[f] + (uint32_t)ks * 1024u));
        }
      }
    };
    load_w(0, wa[0]);
#pragma unroll
    for (int tg = 0; tg < 3; ++tg) {  // dr = tg - 1
      if (tg < 2) load_w(tg + 1, wa[(tg + 1) & 1]);
#pragma unroll
      for (int tt = 0; tt < 3; ++tt) {  // ds = tt - 1
        if (3 * tg + tt < t0 || 3 * tg + tt >= t1) continue;  // wave-uniform
        bf16x8 fb[NPG];
#pragma unroll
        for (int g = 0; g < NPG; ++g) {
          const int rr = brow[g] + tg, cc = bcol[g] + tt;
          fb[g] = *(const bf16x8*)(reg + (rr * RW + cc) * 64 + 16 * (gq ^ ((cc >> 2) & 3)));
        }
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
          for (int g = 0; g < NPG; ++g)
            acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[tg & 1][tt][f], fb[g], acc[f][g], 0, 0, 0);
      }
    }
    if (chunk + 1 < c1) store_x();  // after this wave's reads of the region (LDS ops of a wave stay in order)
  }

  // partial tiles of the 8 waves -> LDS (the regions' bytes: every wave is past its reads)
  __syncthreads();
  f32x4* red = (f32x4*)smem;  // [NWV][NF * NPG][64]
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int g = 0; g < NPG; ++g) red[(wave * NF * NPG + f * NPG + g) * 64 + lane] = acc[f][g];
  __syncthreads();
  const auto ry = make_rsrc(a.y, a.ybytes);
  for (int u = threadIdx.x; u < NF * NPG * 64; u += NWV * 64) {
    const int q = u >> 6, l = u & 63;
    f32x4 v = red[q * 64 + l];
#pragma unroll
    for (int w = 1; w < NWV; ++w) v += red[(w * NF * NPG + q) * 64 + l];
    const int f = q / NPG, g = q - f * NPG;
    const int cl = 16 * f + 4 * (l >> 4);
    const int c = cout0 + cl;
    const float4 sc = *(const float4*)(a.escale + c), sh = *(const float4*)(a.eshift + c);
    float o[4] = {fmaf(v[0], sc.x, sh.x), fmaf(v[1], sc.y, sh.y), fmaf(v[2], sc.z, sh.z), fmaf(v[3], sc.w, sh.w)};
    if (a.erelu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = fmaxf(o[r], 0.f);
    }
    const uint2 pk = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
    const int p = 16 * g + (l & 15);
    const int pr = p / WB, pc = p - pr * WB;
    const int m = ((img * a.H + h0 + pr) << a.wshift) + w0 + pc;
    bstore8(ry, (uint32_t)(m * a.ypitch + c) * 2u, pk);
    if (a.pool) ytile[p][cl >> 2] = pk;
  }
  if (!a.pool) return;  // block-uniform; R == 2 here
  __syncthreads();
  const auto rp = make_rsrc(a.pool, a.pbytes);
  for (int u = threadIdx.x; u < (WB / 2) * (NC / 4); u += NWV * 64) {
    const int wo = u / (NC / 4), cq = u - wo * (NC / 4);
    const int p00 = 2 * wo, p10 = WB + 2 * wo;
    const uint2 qv[4] = {ytile[p00][cq], ytile[p00 + 1][cq], ytile[p10][cq], ytile[p10 + 1][cq]};
    float mx[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t wd = e < 2 ? qv[0].x : qv[0].y;
      mx[e] = __uint_as_float((e & 1) ? (wd & 0xffff0000u) : (wd << 16));
    }
#pragma unroll
    for (int t = 1; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t wd = e < 2 ? qv[t].x : qv[t].y;
        mx[e] = fmaxf(mx[e], __uint_as_float((e & 1) ? (wd & 0xffff0000u) : (wd << 16)));
      }
    const int mo = (img * (a.H >> 1) + (h0 >> 1)) * (a.W >> 1) + (w0 >> 1) + wo;
    bstore8(rp, (uint32_t)(mo * a.ppitch + cout0 + 4 * cq) * 2u, make_uint2(pack2bf(mx[0], mx[1]), pack2bf(mx[2], mx[3])));
  }
}

// ---------------------------------------------------------------------------------------------
// Persistent chain of row-band layers of one map size (layer l + 1's input = layer l's output) in ONE
// launch with row-level readiness counters instead of kernel boundaries (measured
// against the per-layer launches by scripts/rowband_bench.py --chain, profiles/dead_ends.md).
// Work items are dealt by a ticket counter in layer order, so an item only ever waits for items with
// smaller tickets, which are already running: no residency assumption, no deadlock. Hand-off
// (cdna_hip_programming.md Guideline 16): the producer's write-through (sc1) stores -> every wave
// vmcnt(0) -> block barrier -> relaxed agent add on each of its rows' counters (a plain-store + agent
// release form measured slower still: the release writes back the whole XCD L2);
// the consumer: one lane polls the counters of its input rows (relaxed agent loads + s_sleep, bounded:
// on timeout it flags *err and goes on, so a bug cannot hang the GPU) -> agent acquire fence ->
// vmcnt(0) -> block barrier -> plain loads. cnt[0] = ticket, cnt[1 + l * rows + r] = slices of row r of
// layer l written; zeroed by the host before every launch.
struct RowbandChainArgs {
  RowbandArgs L[4];
  int nl;
  int start[5];  // first ticket of each layer
  int nct[4];    // 32-channel slices per layer (a row is complete at nct)
  int rows;      // N * H
  int* cnt;
  int* err;
  int spin_limit;  // polls per row before the wait gives up (RDP_CHAIN_SPINS)
};

// Every branch around a block barrier is wave-uniform: the ticket, the polls and the counter adds are
// issued by ALL lanes of wave 0 (the other lanes add 0; the compiler's atomic combining leaves one add per
// wave instruction) under `wave == 0`, a scalar branch. (A first form with `threadIdx.x == 0` regions
// inside the ticket loop was compiled into a divergent loop whose lanes 1..63 kept re-running the old
// ticket with the other waves while lane 0 waited for them: a hang.)
template <int NF, int NPG, int G>
__global__ __launch_bounds__(512, 4) void conv_rowband_chain_kernel(const RowbandChainArgs c) {
  __shared__ RbSmem<NF, NPG> sm;
  __shared__ int s_ticket;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int one = lane == 0 ? 1 : 0;
  const int total = c.start[c.nl];
  while (true) {
    if (wave == 0) {
      const int v = __hip_atomic_fetch_add(c.cnt, one, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_ticket = __builtin_amdgcn_readfirstlane(v);  // lane 0's value: the ticket
    }
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(s_ticket);
    if (t >= total) break;
    int l = 0;
    while (l + 1 < c.nl && t >= c.start[l + 1]) ++l;
    l = __builtin_amdgcn_readfirstlane(l);
    const RowbandArgs& a = c.L[l];  // uniform index into the kernel arguments: scalar loads
    const int lid = t - c.start[l];
    const int nb = a.N * a.bands;
    const int band = lid - (lid / nb) * nb;
    const int img = band / a.bands, h0 = (band - img * a.bands) * a.R;
    if (l > 0) {  // input rows h0 - 1 .. h0 + R of layer l - 1 complete
      if (wave == 0) {
        const int r0 = max(h0 - 1, 0), r1 = min(h0 + a.R, a.H - 1);
        const int* rc = c.cnt + 1 + (l - 1) * c.rows + img * a.H;
        for (int r = r0; r <= r1; ++r) {
          for (int spins = 0;; ++spins) {
            const int v = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(rc + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (v >= c.nct[l - 1]) break;
            if (spins >= c.spin_limit) {
              __hip_atomic_store(c.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              break;
            }
            __builtin_amdgcn_s_sleep(8);
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
    }
    rowband_tile<NF, NPG, G, true>(a, (uint32_t)lid, sm);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its write-through stores landed
    __syncthreads();
    if (wave == 0) {
      int* rc = c.cnt + 1 + l * c.rows + img * a.H + h0;
      for (int r = 0; r < a.R; ++r) __hip_atomic_fetch_add(rc + r, one, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Operand bytes the kernel moves from L2 (every block re-reads its weight slice; every activation is read
// once per tap and per 32-channel output slice). Measured (scripts/rowband_bench.py, N = 1, MI355X) the
// kernel runs at ~8-9 TB/s of these bytes: it beats the split-K implicit GEMM + reduce pair at <= ~150 MB
// (17-25 % faster on the 64^2 128 -> 256, 32^2 256 -> 512, 16^2 512 -> 512, 32^2 512 -> 256 and
// 64^2 256 -> 128 layers) and loses from ~225 MB up (32^2 1024 -> 512: 64 vs 27 us).
extern "C" long rdp_conv_rowband_bytes(int N, int H, int W, int Cin, int Cout, int pool) {
  const int R = pool && H % 2 == 0 && 2 * W <= 64 ? 2 : 1;
  const long wb = (long)Cout * 9 * Cin * 2, xb = (long)N * H * W * Cin * 2;
  return wb * ((long)N * H / R) + xb * 9 * (Cout / 32);
}

// With the fragment-major weight copy (1 KiB contiguous per MFMA fragment: 8 full lines per load instead of
// 16 half lines) a weight byte costs about half an activation byte (scripts/rowband_bench.py variant 17:
// 16^2 512 -> 512 8.8 vs 14.6 us on OHWI weights, 32^2 256 -> 512 13.2 vs 18.9). The eval dispatch
// (bindings conv_fwd with wfrag) takes the row-band kernel up to 250 MB of weighted operand bytes: every
// <= 64^2 layer of the U-Net but the two long-K decoder convs (32^2 1024 -> 512, 64^2 512 -> 256).
static int ilog2_exact(long v);

// C1 / C2: the two sources' channels (C2 = 0 for one source). Every shape predicate rdp_conv_rowband_ex
// applies is checked here too, so a mode this returns is never rejected by the launch (W and Cin / 32
// powers of two, each source a multiple of 32 channels); the Python executor asks this same function
// (binding rowband_frag_mode) which layers need a fragment-major weight copy.
extern "C" int rdp_conv_rowband_frag_auto(int N, int H, int W, int C1, int C2, int Cout) {
  static const int on = [] {
    const char* e = getenv("RDP_ROWBAND");
    return e ? atoi(e) : 1;
  }();
  const int Cin = C1 + C2;
  if (!on || W < 16 || Cin < 64 || Cout < 64 || Cout % 32 || C1 % 32 || C2 % 32) return 0;
  if (ilog2_exact(W) < 0 || ilog2_exact(Cin / 32) < 0) return 0;
  const long M = (long)N * H * W;
  const long wb = (long)Cout * 9 * Cin * 2, xb = M * Cin * 2;
  static const long xmax = [] {
    const char* e = getenv("RDP_ROWBAND_X_MAXPIX");  // 0 turns the activation-staged kernel off
    return e ? atol(e) : 65536L;  // (the work bound below decides; up3.conv2 at N = 2: 20.0 vs 32.5 us)
  }();
  // (64 input channels stay on the split-K GEMM: 128^2 64 -> 128 18.0 vs 11.5 us, four waves staging one chunk)
  const bool xch = (Cin / 32) % 8 == 0 || Cin == 128;
  if (xch && M <= xmax && W <= 256) {  // activation-staged (x read ~3x instead of 9x)
    // ... while its work (blocks x K, the launch's own tiling below) stays within about two waves of 512
    // blocks: past that the GEMM wins (scripts/rowband_bench.py --batch 1 / 2 / 4, every <= 128^2 layer of
    // the U-Net: e.g. up1.conv1 17.9 vs 26.9 us at N = 1 but 44.9 vs 38.8 at N = 2, down2.conv1 20.9 vs
    // 25.3 at N = 2 but 38.9 vs 20.2 at N = 4; 128-channel inputs, staged in 4 chunks, cross over earlier)
    const int WB = W < 32 ? W : 32, segs = W / WB;
    const bool r2 = H % 2 == 0 && (long)N * (H / 2) * segs * (Cout / 32) >= 256;
    const long blocks = (long)N * (H / (r2 ? 2 : 1)) * segs * (Cout / 32);
    const long work = blocks * 9 * Cin;
    if (work <= ((Cin / 32) % 8 == 0 ? 2500000L : 1300000L)) return 2;
    return 0;
  }
  if (M > 4096 || W > 64) return 0;
  return wb * ((long)N * H) / 2 + xb * 9 * (Cout / 32) <= 250000000L ? 1 : 0;
}

static int ilog2_exact(long v) {
  int s = 0;
  while ((1L << s) < v) ++s;
  return (1L << s) == v ? s : -1;
}

// Returns 1 if it also wrote the pool, 0 if not, < 0 (nothing launched) when the shape does not fit.
// wfrag: w is the fragment-major copy of the OHWI weights (rdp_rowband_frag_weights) instead of OHWI.
extern "C" int rdp_conv_rowband_ex(const void* x1, const void* x2, long xbytes1, long xbytes2, int C1, int C2,
                                   int pitch1, int pitch2, const void* w, long wbytes, int ldw, void* y, long ybytes,
                                   int ypitch, int N, int H, int W, int Cout, const float* escale, const float* eshift,
                                   int erelu, void* pool, long pbytes, int ppitch, int wfrag, hipStream_t s);
extern "C" int rdp_conv_rowband(const void* x1, const void* x2, long xbytes1, long xbytes2, int C1, int C2, int pitch1,
                                int pitch2, const void* w, long wbytes, int ldw, void* y, long ybytes, int ypitch, int N,
                                int H, int W, int Cout, const float* escale, const float* eshift, int erelu, void* pool,
                                long pbytes, int ppitch, hipStream_t s) {
  return rdp_conv_rowband_ex(x1, x2, xbytes1, xbytes2, C1, C2, pitch1, pitch2, w, wbytes, ldw, y, ybytes, ypitch, N, H,
                             W, Cout, escale, eshift, erelu, pool, pbytes, ppitch, 0, s);
}

extern "C" int rdp_conv_rowband_ex(const void* x1, const void* x2, long xbytes1, long xbytes2, int C1, int C2,
                                   int pitch1, int pitch2, const void* w, long wbytes, int ldw, void* y, long ybytes,
                                   int ypitch, int N, int H, int W, int Cout, const float* escale, const float* eshift,
                                   int erelu, void* pool, long pbytes, int ppitch, int wfrag, hipStream_t s) {
  const int Cin = C1 + C2;
  const int cs = ilog2_exact(Cin / 32), ws = ilog2_exact(W);
  if (C1 % 32 || C2 % 32 || Cin < 64 || Cin % 32 || cs < 0 || ws < 4 || W > (wfrag == 2 ? 256 : 64) || Cout % 32)
    return -1;
  if (!escale || !eshift || (!wfrag && ldw < 9 * Cin) || (wfrag && wbytes < (long)Cout * 9 * Cin * 2) || (C2 && !x2))
    return -1;
  if (pitch1 % 8 || (C2 && pitch2 % 8) || ypitch % 4) return -1;
  if (xbytes1 >= (1L << 31) || xbytes2 >= (1L << 31) || wbytes >= (1L << 31) || ybytes >= (1L << 31) ||
      pbytes >= (1L << 31))
    return -1;
  if (wfrag == 2) {  // the activation-staged kernel: 32-channel chunks (a multiple of 8, or 2 / 4)
    if ((Cin / 32) % 8 && Cin != 64 && Cin != 128) return -1;
    const int WB = W < 32 ? W : 32;
    const bool plx = pool != nullptr && H % 2 == 0 && ppitch % 4 == 0;
    // two-row tiles (each block's weight slice serves twice the pixels) wherever that grid still has >= 256
    // blocks: up1.conv1 22.4 -> 18.2 us, up2.conv1 24.5 -> 21.9, down3.conv1 7.8 -> 6.9 (at 128 blocks, the
    // 16^2 and 32^2 -> 256 convs, one-row tiles stay faster); RDP_ROWBAND_R2=0 keeps one-row tiles (A/B)
    static const int r2_on = [] {
      const char* e = getenv("RDP_ROWBAND_R2");
      return e ? atoi(e) : 1;
    }();
    const bool r2 = r2_on && H % 2 == 0 && (long)N * (H / 2) * (W / (W < 32 ? W : 32)) * (Cout / 32) >= 256;
    const int Rx = plx || r2 ? 2 : 1;
    RowbandArgs a;
    a.x1 = (const u16*)x1; a.x2 = (const u16*)x2;
    a.xbytes1 = (uint32_t)xbytes1; a.xbytes2 = (uint32_t)xbytes2;
    a.C1 = C1; a.C2 = C2; a.pitch1 = pitch1; a.pitch2 = pitch2;
    a.w = (const u16*)w; a.wbytes = (uint32_t)wbytes; a.ldw = ldw;
    a.y = (u16*)y; a.ybytes = (uint32_t)ybytes; a.ypitch = ypitch;
    a.pool = plx ? (u16*)pool : nullptr; a.pbytes = plx ? (uint32_t)pbytes : 0u; a.ppitch = ppitch;
    a.escale = escale; a.eshift = eshift; a.erelu = erelu;
    a.N = N; a.H = H; a.W = W; a.Cout = Cout; a.wshift = ws;
    a.R = Rx; a.bands = H / Rx; a.cshift = cs; a.T = 9 * Cin / 32; a.wfrag = 1; a.segs = W / WB;
    const int grid = N * a.bands * a.segs * (Cout / 32);
    const int PBx = Rx * WB;
    if (PBx == 16) hipLaunchKernelGGL((conv_rowband_x_kernel<1, 1>), dim3(grid), dim3(512), 0, s, a);
    else if (PBx == 32 && Rx == 1) hipLaunchKernelGGL((conv_rowband_x_kernel<2, 1>), dim3(grid), dim3(512), 0, s, a);
    else if (PBx == 32) hipLaunchKernelGGL((conv_rowband_x_kernel<2, 2>), dim3(grid), dim3(512), 0, s, a);
    else if (PBx == 64) hipLaunchKernelGGL((conv_rowband_x_kernel<4, 2>), dim3(grid), dim3(512), 0, s, a);
    else return -1;
    return plx ? 1 : 0;
  }
  // the pool needs two rows per block: only where that block is <= 64 pixels (else the caller pools)
  const bool pl = pool != nullptr && H % 2 == 0 && ppitch % 4 == 0 && 2 * W <= 64;
  const int R = pl ? 2 : 1;
  const int PB = R * W;
  RowbandArgs a;
  a.x1 = (const u16*)x1; a.x2 = (const u16*)x2;
  a.xbytes1 = (uint32_t)xbytes1; a.xbytes2 = (uint32_t)xbytes2;
  a.C1 = C1; a.C2 = C2; a.pitch1 = pitch1; a.pitch2 = pitch2;
  a.w = (const u16*)w; a.wbytes = (uint32_t)wbytes; a.ldw = ldw;
  a.y = (u16*)y; a.ybytes = (uint32_t)ybytes; a.ypitch = ypitch;
  a.pool = pl ? (u16*)pool : nullptr; a.pbytes = pl ? (uint32_t)pbytes : 0u; a.ppitch = ppitch;
  a.escale = escale; a.eshift = eshift; a.erelu = erelu;
  a.N = N; a.H = H; a.W = W; a.Cout = Cout; a.wshift = ws;
  a.R = R; a.bands = H / R; a.cshift = cs; a.T = 9 * Cin / 32; a.wfrag = wfrag;
  const int grid = N * a.bands * (Cout / 32);
  if (PB == 16) hipLaunchKernelGGL((conv_rowband_kernel<2, 1, 4>), dim3(grid), dim3(512), 0, s, a);
  else if (PB == 32) hipLaunchKernelGGL((conv_rowband_kernel<2, 2, 2>), dim3(grid), dim3(512), 0, s, a);
  else if (PB == 64) hipLaunchKernelGGL((conv_rowband_kernel<2, 4, 1>), dim3(grid), dim3(512), 0, s, a);
  else return -1;
  return pl ? 1 : 0;
}

// The chain launch: layer 0 reads x (C0 channels), layer l > 0 reads layer l - 1's output; every layer is
// an eval conv (BN folded + ReLU) on the same N x H x W map. cnt: >= 1 + nl * N * H ints, err: 1 int.
// Returns 0, or < 0 (nothing launched) when a layer does not fit the row-band kernel.
extern "C" int rdp_conv_rowband_chain(int nl, const void* x, long xbytes, int C0, int xpitch, const void* const* w,
                                      const long* wbytes, const int* ldw, void* const* y, const long* ybytes,
                                      const int* ypitch, const int* cout, const float* const* escale,
                                      const float* const* eshift, int N, int H, int W, int* cnt, int* err,
                                      hipStream_t s) {
  if (nl < 1 || nl > 4) return -1;
  const int ws = ilog2_exact(W);
  if (ws < 4 || W != 16) return -1;  // one tile shape (16-pixel rows) for the whole chain
  RowbandChainArgs c;
  c.nl = nl;
  c.rows = N * H;
  c.cnt = cnt;
  c.err = err;
  static const int spins = [] {
    const char* e = getenv("RDP_CHAIN_SPINS");
    return e ? atoi(e) : (1 << 20);
  }();
  c.spin_limit = spins;
  c.start[0] = 0;
  int cin = C0;
  for (int l = 0; l < nl; ++l) {
    const int cs = ilog2_exact(cin / 32);
    if (cin % 32 || cin < 64 || cs < 0 || cout[l] % 32 || ldw[l] < 9 * cin || ypitch[l] % 4) return -1;
    RowbandArgs& a = c.L[l];
    a.x1 = (const u16*)(l == 0 ? x : y[l - 1]);
    a.x2 = nullptr;
    a.xbytes1 = (uint32_t)(l == 0 ? xbytes : ybytes[l - 1]);
    a.xbytes2 = 0;
    a.C1 = cin; a.C2 = 0; a.pitch1 = l == 0 ? xpitch : ypitch[l - 1]; a.pitch2 = 0;
    a.w = (const u16*)w[l]; a.wbytes = (uint32_t)wbytes[l]; a.ldw = ldw[l];
    a.y = (u16*)y[l]; a.ybytes = (uint32_t)ybytes[l]; a.ypitch = ypitch[l];
    a.pool = nullptr; a.pbytes = 0; a.ppitch = 0;
    a.escale = escale[l]; a.eshift = eshift[l]; a.erelu = 1;
    a.N = N; a.H = H; a.W = W; a.Cout = cout[l]; a.wshift = ws;
    a.R = 1; a.bands = H; a.cshift = cs; a.T = 9 * cin / 32; a.wfrag = 0;
    c.nct[l] = cout[l] / 32;
    c.start[l + 1] = c.start[l] + N * H * c.nct[l];
    cin = cout[l];
  }
  for (int l = nl; l < 4; ++l) c.L[l] = c.L[0];
  const int grid = std::min(c.start[nl], 512);
  if (hipMemsetAsync(cnt, 0, (size_t)(1 + nl * c.rows) * sizeof(int), s) != hipSuccess) return -2;
  hipLaunchKernelGGL((conv_rowband_chain_kernel<2, 1, 3>), dim3(grid), dim3(512), 0, s, c);
  return 0;
}

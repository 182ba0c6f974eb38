// Convolution weight gradient, NHWC bf16 in, fp32 out; MFMA 16x16x32 over pixels.
//
// Replaces the cuDNN/MIOpen wgrad that autograd launches for every nn.Conv2d of the reference
// U-Net (/root/reference/scripts/train_segmenter.py:162 loss.backward()).
//
// GEMM view: dW^T[col = (tap, cin)][cout] = sum_pixels im2col(x)[pix][col] * dY[pix][cout].
// The reduction (pixel) axis is the strided one in NHWC, so both operand tiles are staged as
// natural [64 pixels][64 channels] rows by LDS-DMA (zero halo via out-of-range offsets) and read
// as MFMA fragments with ds_read_b64_tr_b16 (hardware transpose). The 16-B chunk of each LDS row
// is XOR-swizzled on the SOURCE address (LDS-DMA writes lane-linear) with a swizzle that makes the
// transposed reads bank-conflict free (derived by simulation; see tests/test_lds_swizzle.py).
//
// Block = 4 waves; wave w owns col-subtile w (64 (tap,cin) columns) x 64 output channels.
// Split-K over pixels; each split writes an fp32 slab [split][Cout][ncols_pad]; rdp_wgrad_reduce
// sums the splits into the parameter-gradient layout (OHWI, i.e. channels_last OIHW).
//
// Measured dead ends (kept out of the code, numbers from scripts/conv_microbench.py at bs32):
//   * STAGES=3 (one block/CU) and BKP=32 variants: slower than (64, 2) on every layer.
//   * software L2 prefetch with 4-B-per-lane loads one line per lane: 1.7x SLOWER (64 distinct
//     lines per wave-instruction saturate the address path, MI355X_MICROARCH.md "access shape").
//   * DMA issue moved between the MFMA halves: slower (DMA latency matters more than VALU slots).
//   * 3-wave blocks (192 columns: no padding for Cin = 64 / 128): +3 % at Cin = 64, -5 % at 128 --
//     the padded MFMAs are not on the critical path of this latency-bound loop.
// PMC (256^2 x 64ch): ~48 % of wave cycles in s_waitcnt/barrier, i.e. latency-bound on x/dY
// streamed from HBM with only one K step of lookahead.
#include "common.h"
#include <algorithm>

struct WgradArgs {
  const u16* x1;
  const u16* x2;
  uint32_t xbytes1, xbytes2;
  int C1, C2, pitch1, pitch2;
  const u16* dy;
  uint32_t dybytes;
  int dypitch;
  float* slab;
  int H, W, M, Cout, Cin;
  int taps, packed;
  int ncols, ncols_pad;
  int colTiles, coutTiles, splits;
  int pix_per_split;
  uint32_t fw_m, fw_s, fh_m, fh_s;  // fast div by W and by H
};

RDP_DEV int swz(int p) { return (((p >> 1) & 1) << 1) | (((p >> 3) & 1) << 2); }

RDP_DEV uint32_t fdiv2(uint32_t n, uint32_t m, uint32_t s) { return (__umulhi(n, m) + n) >> s; }

// BKP pixels per K step (64 or 32), STAGES LDS buffers (STAGES-1 steps in flight under the MFMAs).
// NWV = 4: wave w owns x-subtile w (64 columns) x 64 couts; NWV = 8: waves 2s, 2s+1 split
// x-subtile s into two 32-column halves (twice the waves per SIMD, same LDS footprint).
template <bool PACKED, bool TILE_FAST, int BKP, int STAGES, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, 2) void conv_wgrad_kernel(const WgradArgs a) {
  constexpr int SUB = BKP * 128;        // one [BKP pixels][64 ch] bf16 tile
  constexpr int BUF = 5 * SUB;          // 4 x-subtiles + 1 dy tile
  constexpr int PIECES = BKP / 8;       // 8-row DMA pieces per subtile
  constexpr int PPW = PIECES / NWV;     // pieces (row groups) per wave
  constexpr int NI = 4 * 4 / NWV;       // 16-column x fragments per wave (4 or 2)
  static_assert(PPW >= 1, "BKP too small for the wave count");
  __shared__ __attribute__((aligned(16))) char smem[STAGES * BUF];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  const uint32_t nwg = gridDim.x;
  const uint32_t lid = xcd_remap(blockIdx.x, nwg);
  // TILE_FAST: consecutive logical ids (same XCD after the remap) = different weight tiles of the
  // SAME pixel range, so they share the dY / X lines in that XCD's L2.
  const int ntiles = a.colTiles * a.coutTiles;
  const int split = TILE_FAST ? lid / ntiles : lid % a.splits;
  const int tile = TILE_FAST ? lid % ntiles : lid / a.splits;
  const int tc = tile % a.colTiles, tn = tile / a.colTiles;
  const int cout0 = tn * 64;
  const int pbeg = split * a.pix_per_split;
  const int pend = min(a.M, pbeg + a.pix_per_split);
  const int nks = (pend - pbeg + BKP - 1) / BKP;

  const auto rx1 = make_rsrc(a.x1, a.xbytes1);
  const auto rx2 = make_rsrc(a.x2 ? a.x2 : a.x1, a.x2 ? a.xbytes2 : 0u);
  const auto rdy = make_rsrc(a.dy, a.dybytes);

  // per-subtile (tap, channel offset, source) -- uniform
  int s_dr[4], s_ds[4], s_ch[4], s_src[4], s_ok[4];
#pragma unroll
  for (int sub = 0; sub < 4; ++sub) {
    const int kc = tc * 256 + sub * 64;
    s_ok[sub] = kc < a.ncols;
    if (PACKED) {
      s_dr[sub] = 0; s_ds[sub] = 0; s_ch[sub] = kc / 8; s_src[sub] = 0;  // s_ch = first tap
    } else {
      const int tap = kc / a.Cin;
      const int cin0 = kc - tap * a.Cin;
      s_dr[sub] = a.taps == 9 ? tap / 3 - 1 : 0;
      s_ds[sub] = a.taps == 9 ? tap % 3 - 1 : 0;
      s_src[sub] = cin0 >= a.C1;
      s_ch[sub] = s_src[sub] ? cin0 - a.C1 : cin0;
    }
  }

  const int rowl = lane >> 3;  // pixel row within an 8-row DMA piece
  const int cpos = lane & 7;   // 16-B position within the LDS row

  auto issue = [&](int ks, char* buf) {
#pragma unroll
    for (int t = 0; t < PPW; ++t) {
      const int s = wave * PPW + t;  // DMA piece index (8 pixel rows)
      const int p = s * 8 + rowl;  // pixel row in the BKP-pixel K step
      const int g = cpos ^ swz(p);  // global 16-B chunk this lane fetches
      const int m = pbeg + ks * BKP + p;
      const bool mv = m < pend;
      const uint32_t q = fdiv2((uint32_t)m, a.fw_m, a.fw_s);
      const int w = m - (int)q * a.W;
      const int h = (int)q - (int)fdiv2(q, a.fh_m, a.fh_s) * a.H;
      // dY piece
      {
        const uint32_t off = mv ? (uint32_t)(m * a.dypitch + cout0 + g * 8) * 2u : RDP_OOB;
        dma16(rdy, (lds_void*)(buf + 4 * SUB + s * 1024), off);
      }
#pragma unroll
      for (int sub = 0; sub < 4; ++sub) {
        int dr = s_dr[sub], ds = s_ds[sub], ch;
        if constexpr (PACKED) {
          const int tap = s_ch[sub] + g;
          dr = tap / 3 - 1; ds = tap % 3 - 1;
          ch = 0;
          const int hh = h + dr, ww = w + ds;
          const bool ok = mv & (bool)s_ok[sub] & (tap < 9) & inb(hh, a.H) & inb(ww, a.W);
          const uint32_t off = ok ? (uint32_t)((m + dr * a.W + ds) * a.pitch1) * 2u : RDP_OOB;
          dma16(rx1, (lds_void*)(buf + sub * SUB + s * 1024), off);
        } else {
          ch = s_ch[sub] + g * 8;
          const int hh = h + dr, ww = w + ds;
          const bool ok = mv & (bool)s_ok[sub] & inb(hh, a.H) & inb(ww, a.W);
          const int pitch = s_src[sub] ? a.pitch2 : a.pitch1;
          const uint32_t off = ok ? (uint32_t)((m + dr * a.W + ds) * pitch + ch) * 2u : RDP_OOB;
          dma16(s_src[sub] ? rx2 : rx1, (lds_void*)(buf + sub * SUB + s * 1024), off);
        }
      }
    }
  };

  f32x4 acc[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane geometry: lane = 16g + 4q + pp
  const int tg = lane >> 4, tq = (lane >> 2) & 3, tpp = lane & 3;

  // one barrier per K step: wait for stage ks (STAGES-2 younger stages stay in flight), the
  // barrier retires every wave's reads of the buffer about to be refilled, then issue ks+STAGES-1.
  constexpr int DMA_PER_STAGE = PPW * 5;
#pragma unroll
  for (int st = 0; st < STAGES - 1; ++st)
    if (st < nks) issue(st, smem + st * BUF);
  for (int ks = 0; ks < nks; ++ks) {
    if constexpr (STAGES == 3) {
      if (ks + 1 < nks) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(DMA_PER_STAGE) : "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    raw_barrier();
    if (ks + STAGES - 1 < nks) issue(ks + STAGES - 1, smem + ((ks + STAGES - 1) % STAGES) * BUF);
    const char* cur = smem + (ks % STAGES) * BUF;
    const int xsub = NWV == 4 ? wave : (wave >> 1);
    const int i0 = NWV == 4 ? 0 : (wave & 1) * NI;  // first 16-column group of this wave
    const char* xb = cur + xsub * SUB;
    const char* db = cur + 4 * SUB;
#pragma unroll
    for (int hf = 0; hf < BKP / 32; ++hf) {
      bf16x8 fa[NI], fb[4];
      const int p0 = 32 * hf + 8 * tg + tq;
      const int sw0 = swz(p0), sw1 = swz(p0 + 4);
      const int ro0 = p0 * 128 + 8 * (tpp & 1), ro1 = ro0 + 4 * 128;
      typedef __attribute__((address_space(3))) bf16x4 lds_v4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 2 * i + (tpp >> 1);
        const int o0 = ro0 + 16 * (c ^ sw0), o1 = ro1 + 16 * (c ^ sw1);
        const bf16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(db + o0));
        const bf16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(db + o1));
        fb[i] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int c = 2 * (i0 + i) + (tpp >> 1);
        const int o0 = ro0 + 16 * (c ^ sw0), o1 = ro1 + 16 * (c ^ sw1);
        const bf16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(xb + o0));
        const bf16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(xb + o1));
        fa[i] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }

  // acc[i][j][r]: col = colbase + 16i + 4*(lane>>4) + r ; cout = cout0 + 16j + (lane&15)
  const int colbase = NWV == 4 ? tc * 256 + wave * 64 : tc * 256 + (wave >> 1) * 64 + (wave & 1) * 32;
  if (colbase >= a.ncols_pad) return;
  const auto rs = make_rsrc(a.slab, (uint32_t)min((long)a.splits * a.Cout * a.ncols_pad * 4l, (long)0x7fffffff));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int co = cout0 + 16 * j + (lane & 15);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int col = colbase + 16 * i + 4 * (lane >> 4);
      const uint32_t off = (uint32_t)(((long)split * a.Cout + co) * a.ncols_pad + col) * 4u;
      uint4 v;
      v.x = __float_as_uint(acc[i][j][0]); v.y = __float_as_uint(acc[i][j][1]);
      v.z = __float_as_uint(acc[i][j][2]); v.w = __float_as_uint(acc[i][j][3]);
      bstore16(rs, off, v);
    }
  }
}

// out[cout][tap][cin_real] (+)= sum_split slab[split][cout][tap*cin_pad + cin]
__global__ void wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out, int splits, int Cout,
                                    int ncols_pad, int taps, int cin_pad, int cin_real, int accumulate) {
  const long total = (long)Cout * taps * cin_real;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int cin = idx % cin_real;
    const long t2 = idx / cin_real;
    const int tap = t2 % taps;
    const int co = t2 / taps;
    const long col = (long)tap * cin_pad + cin;
    // 8 independent accumulators: the split loop is latency-bound otherwise (hundreds of splits)
    const float* p = slab + (long)co * ncols_pad + col;
    const long stride = (long)Cout * ncols_pad;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f, s5 = 0.f, s6 = 0.f, s7 = 0.f;
    int sp = 0;
    for (; sp + 8 <= splits; sp += 8) {
      s0 += p[(sp + 0) * stride]; s1 += p[(sp + 1) * stride]; s2 += p[(sp + 2) * stride]; s3 += p[(sp + 3) * stride];
      s4 += p[(sp + 4) * stride]; s5 += p[(sp + 5) * stride]; s6 += p[(sp + 6) * stride]; s7 += p[(sp + 7) * stride];
    }
    for (; sp < splits; ++sp) s0 += p[sp * stride];
    const float s = ((s0 + s1) + (s2 + s3)) + ((s4 + s5) + (s6 + s7));
    out[idx] = accumulate ? out[idx] + s : s;
  }
}

extern "C" int rdp_conv_wgrad(const void* x1, const void* x2, long xbytes1, long xbytes2, int C1, int C2, int pitch1,
                              int pitch2, const void* dy, long dybytes, int dypitch, float* slab, long slab_elems,
                              float* out, int accumulate, int N, int H, int W, int Cout, int taps, int packed,
                              int cin_real, int splits, int variant, hipStream_t s) {
  WgradArgs a;
  a.x1 = (const u16*)x1; a.x2 = (const u16*)x2;
  a.xbytes1 = (uint32_t)xbytes1; a.xbytes2 = (uint32_t)xbytes2;
  a.C1 = C1; a.C2 = C2; a.pitch1 = pitch1; a.pitch2 = pitch2;
  a.dy = (const u16*)dy; a.dybytes = (uint32_t)dybytes; a.dypitch = dypitch;
  a.slab = slab; a.H = H; a.W = W; a.M = N * H * W; a.Cout = Cout;
  a.taps = taps; a.packed = packed;
  if (packed) {
    if (C1 != 8 || C2 != 0 || taps != 9) return -1;
    a.Cin = 8; a.ncols = 72;
  } else {
    if (C1 % 64 || C2 % 64) return -1;
    a.Cin = C1 + C2; a.ncols = taps * a.Cin;
  }
  if (Cout % 64) return -1;
  if (xbytes1 >= (1l << 31) || xbytes2 >= (1l << 31) || dybytes >= (1l << 31)) return -1;
  a.colTiles = (a.ncols + 255) / 256;
  a.ncols_pad = a.colTiles * 256;
  a.coutTiles = Cout / 64;
  if (splits < 1) splits = 1;
  int pps = (a.M + splits - 1) / splits;
  pps = (pps + 63) / 64 * 64;
  a.pix_per_split = pps;
  a.splits = (a.M + pps - 1) / pps;
  if ((long)a.splits * Cout * a.ncols_pad > slab_elems) return -2;
  if ((long)a.splits * Cout * a.ncols_pad * 4l >= (1l << 31)) return -3;
  FastDiv fw = make_fastdiv(W), fh = make_fastdiv(H);
  a.fw_m = fw.m; a.fw_s = fw.s; a.fh_m = fh.m; a.fh_s = fh.s;
  const int nblk = a.colTiles * a.coutTiles * a.splits;
  if (packed) {
    hipLaunchKernelGGL((conv_wgrad_kernel<true, true, 64, 2, 8>), dim3(nblk), dim3(512), 0, s, a);
  } else if (variant == 1) {  // alternatives kept for the microbenchmark (measured slower on gfx950)
    hipLaunchKernelGGL((conv_wgrad_kernel<false, true, 32, 3>), dim3(nblk), dim3(256), 0, s, a);
  } else if (variant == 2) {
    hipLaunchKernelGGL((conv_wgrad_kernel<false, true, 64, 3>), dim3(nblk), dim3(256), 0, s, a);
  } else if (variant == 3) {  // 4-wave blocks (previous default)
    hipLaunchKernelGGL((conv_wgrad_kernel<false, true, 64, 2, 4>), dim3(nblk), dim3(256), 0, s, a);
  } else {  // default: BK=64 pixels per stage, double-buffered, 8 waves (64 couts x 32 columns each)
    hipLaunchKernelGGL((conv_wgrad_kernel<false, true, 64, 2, 8>), dim3(nblk), dim3(512), 0, s, a);
  }
  const int creal = packed ? cin_real : a.Cin;
  const long total = (long)Cout * taps * creal;
  const int rb = (int)std::min<long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(rb), dim3(256), 0, s, slab, out, a.splits, Cout, a.ncols_pad, taps,
                     packed ? 8 : a.Cin, creal, accumulate);
  return a.splits;
}

// Slab size needed (elements) for a given configuration.
extern "C" long rdp_conv_wgrad_slab_elems(int N, int H, int W, int Cin, int Cout, int taps, int packed, int splits) {
  const int ncols = packed ? 72 : taps * Cin;
  const int ncols_pad = (ncols + 255) / 256 * 256;
  const long M = (long)N * H * W;
  long pps = (M + splits - 1) / splits;
  pps = (pps + 63) / 64 * 64;
  const long sp = (M + pps - 1) / pps;
  return sp * Cout * ncols_pad;
}

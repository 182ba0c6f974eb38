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
#include <stdlib.h>
#include <string.h>

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
  // UTR (ConvTranspose2d(2, s2) weight gradient, rdp_conv_wgrad_upT): x1 = the output gradient du
  // [N][uH2][uW2][C1], read at the 4 sub-pixels (2h + tap/2 + uoy, 2w + tap%2 + uox) of low-res
  // pixel (h, w) -- the "taps" -- instead of an unshuffled [N][h][w][4 C1] copy
  int uH2 = 0, uW2 = 0, uoy = 0, uox = 0;
};

RDP_DEV int swz(int p) { return (((p >> 1) & 1) << 1) | (((p >> 3) & 1) << 2); }

RDP_DEV uint32_t fdiv2(uint32_t n, uint32_t m, uint32_t s) { return (__umulhi(n, m) + n) >> s; }

// BKP = 64 pixels per K step, double-buffered; 8 waves: waves 2s, 2s+1 split x-subtile s into two
// 32-column halves (twice the waves per SIMD of a 4-wave block, same LDS footprint).
template <bool PACKED, bool UTR = false>
__global__ __launch_bounds__(512, 2) void conv_wgrad_kernel(const WgradArgs a) {
  constexpr bool TILE_FAST = true;
  constexpr int BKP = 64, STAGES = 2, NWV = 8;
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
      s_dr[sub] = UTR ? tap >> 1 : a.taps == 9 ? tap / 3 - 1 : 0;
      s_ds[sub] = UTR ? tap & 1 : a.taps == 9 ? tap % 3 - 1 : 0;
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
        dma16_async(rdy, (lds_void*)(buf + 4 * SUB + s * 1024), off);
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
          dma16_async(rx1, (lds_void*)(buf + sub * SUB + s * 1024), off);
        } else if constexpr (UTR) {  // sub-pixel (dr, ds) of the (2h + uoy, 2w + uox) pixel of du
          ch = s_ch[sub] + g * 8;
          const int img = (int)fdiv2(q, a.fh_m, a.fh_s);
          const int px = (img * a.uH2 + 2 * h + a.uoy + dr) * a.uW2 + 2 * w + a.uox + ds;
          const uint32_t off = mv & (bool)s_ok[sub] ? (uint32_t)(px * a.pitch1 + ch) * 2u : RDP_OOB;
          dma16_async(rx1, (lds_void*)(buf + sub * SUB + s * 1024), off);
        } else {
          ch = s_ch[sub] + g * 8;
          const int hh = h + dr, ww = w + ds;
          const bool ok = mv & (bool)s_ok[sub] & inb(hh, a.H) & inb(ww, a.W);
          const int pitch = s_src[sub] ? a.pitch2 : a.pitch1;
          const uint32_t off = ok ? (uint32_t)((m + dr * a.W + ds) * pitch + ch) * 2u : RDP_OOB;
          dma16_async(s_src[sub] ? rx2 : rx1, (lds_void*)(buf + sub * SUB + s * 1024), off);
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

// ---------------------------------------------------------------------------------------------
// Halo-reuse weight gradient for 3x3 convs whose pixels split into 64-pixel segments of whole rows
// or of one row (W % 64 == 0, or W | 64 with H * W % 64 == 0: every U-Net layer at 256^2..16^2).
//
// The generic kernel above stages one [64 px][64 ch] x tile per (tap, cin-chunk) column subtile,
// i.e. the same input pixels 9 times (once per tap) and 40 KB of DMA per 2 MFLOP. Here one K step
// is one 64-pixel segment (h, w0..w0+63) of one image (or 64 / W whole rows), and the block owns ALL 9 taps of one
// 64-channel input chunk: it stages the three input rows h-1, h, h+1 over pixels w0-1 .. w0+64
// (66 used of 72 staged rows per region, zero halo from out-of-range offsets) plus the dY segment,
// and every tap (dr, ds) is a row-shifted window (rows ds+1 .. ds+64 of region dr+1) of that one
// image. Per K step: 27 KB of x + 8 KB per 64 couts of dY for 9 x 64 x BN x 64 MACs (2.7x the
// FLOP per staged byte at BN = 64, 3.4x at BN = 128).
//
// Block = BN/16 waves; wave w owns input channels 16*(w&3) .. +15 of the chunk for all 9 taps and
// output channels 64*(w>>2) .. +63: 9 x 4 MFMA 16x16x32 accumulators (144 VGPRs), A fragments by
// ds_read_b64_tr_b16 from the shifted windows, B fragments from the dY tile (same LDS image and
// swizzle as the generic kernel). Split-K over row segments into the same fp32 slab format, reduced
// by wgrad_reduce_kernel.
struct WgradHaloArgs {
  const u16* x1;
  const u16* x2;
  uint32_t xbytes1, xbytes2;
  int C1, C2, pitch1, pitch2;
  const u16* dy;
  uint32_t dybytes;
  int dypitch;
  float* slab;
  uint32_t slab_bytes;
  int H, W, Cout, ncols;  // ncols = 9 * Cin = slab row length
  int cinTiles, coutTiles, splits, segs_per_split, nseg;
  uint32_t fw_m, fw_s, fh_m, fh_s;
};

// (Measured dead ends, numbers in profiles/dead_ends.md: a staggered two-group schedule and a 3-stage
// ring of this kernel; ablations: the DMA stream and the MFMA / LDS-read work each take ~70 % of the
// kernel but barely overlap -- the reason conv_wgrad_pp.hip exists.)
template <int BN, bool MULTIROW>
__global__ __launch_bounds__(BN * 4, 2) void conv_wgrad_halo_kernel(const WgradHaloArgs a) {
  constexpr int STAGES = 2;
  constexpr int NWV = BN / 16;
  constexpr int XREG = 72 * 128;                  // one staged input row region (72 pixel rows x 64 ch)
  constexpr int DSUB = 64 * 128;                  // one [64 px][64 cout] dY subtile
  constexpr int BUF = 3 * XREG + (BN / 64) * DSUB;
  constexpr int XPIECES = 27, NPIECES = XPIECES + 8 * (BN / 64);
  constexpr int PPW = (NPIECES + NWV - 1) / NWV;  // DMA pieces (8 rows x 128 B) per wave per stage
  __shared__ __attribute__((aligned(16))) char smem[STAGES * BUF];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  const uint32_t lid = xcd_remap(blockIdx.x, gridDim.x);
  // consecutive logical ids (one XCD) = different weight tiles of the same segment range: they
  // share the dY / x lines in that XCD's L2
  const int ntiles = a.cinTiles * a.coutTiles;
  const int split = lid / ntiles, tile = lid - split * ntiles;
  const int tc = tile % a.cinTiles, tn = tile / a.cinTiles;
  const int cin0 = tc * 64, cout0 = tn * BN;
  const int s0 = split * a.segs_per_split;
  const int s1 = min(a.nseg, s0 + a.segs_per_split);
  const int nks = s1 - s0;

  const bool src2 = cin0 >= a.C1;
  const auto rx = src2 ? make_rsrc(a.x2, a.xbytes2) : make_rsrc(a.x1, a.xbytes1);
  const int pitch = src2 ? a.pitch2 : a.pitch1;
  const int ch0 = src2 ? cin0 - a.C1 : cin0;
  const auto rdy = make_rsrc(a.dy, a.dybytes);

  const int rowl = lane >> 3, cpos = lane & 7;

  auto issue = [&](int ks, char* buf) {
    const int m0 = (s0 + ks) * 64;  // first pixel of the segment
    const uint32_t q = fdiv2((uint32_t)m0, a.fw_m, a.fw_s);
    const int w0 = m0 - (int)q * a.W;
    const int h = (int)q - (int)fdiv2(q, a.fh_m, a.fh_s) * a.H;
#pragma unroll
    for (int t = 0; t < PPW; ++t) {
      const int piece = wave + t * NWV;  // wave-uniform
      if (piece < XPIECES) {
        const int r = piece / 9, pj = piece - r * 9;  // region (dr + 1), 8-row piece in the region
        const int j = pj * 8 + rowl;                  // staged row: pixel w0 - 1 + j of image row h + dr
        const int g = cpos ^ swz(j);
        // image row of the staged pixel: row h + dr + floor((w0 - 1 + j) / W). Wide rows (W >= 64)
        // keep only pixels of row h + dr (the rest is the zero halo); multi-row segments (W | 64)
        // keep every in-image row and mask the row-crossing taps on the dY side instead.
        const int wj = w0 - 1 + j;
        const int wq = wj < 0 ? -1 : (int)fdiv2((uint32_t)wj, a.fw_m, a.fw_s);
        const bool ok = (j < 66) & (MULTIROW || wq == 0) & inb(h + r - 1 + wq, a.H);
        const uint32_t off = ok ? (uint32_t)((m0 + (r - 1) * a.W + j - 1) * pitch + ch0 + g * 8) * 2u : RDP_OOB;
        dma16_async(rx, (lds_void*)(buf + r * XREG + pj * 1024), off);
      } else if (piece < NPIECES) {
        const int d = piece - XPIECES, sub = d >> 3, pj = d & 7;
        const int p = pj * 8 + rowl;
        const int g = cpos ^ swz(p);
        const uint32_t off = (uint32_t)((m0 + p) * a.dypitch + cout0 + sub * 64 + g * 8) * 2u;
        dma16_async(rdy, (lds_void*)(buf + 3 * XREG + sub * DSUB + pj * 1024), off);
      }
    }
  };

  f32x4 acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane geometry (see conv_wgrad_kernel): lane = 16 tg + 4 tq + tpp
  const int tg = lane >> 4, tq = (lane >> 2) & 3, tpp = lane & 3;
  const int cf = wave & 3, cg = wave >> 2;
  const int ca = 2 * cf + (tpp >> 1);  // 16-B chunk of this lane's A fragment row (input channels)
  typedef __attribute__((address_space(3))) bf16x4 lds_v4;
  // LDS fragment offsets, hoisted: the swizzle reads pixel-row bits 1 and 3 only, so the half step's
  // 32-row offset (hf) is a constant 4 KB -- one set of lane offsets serves both halves (immediates)
  const int q0 = 8 * tg + tq;
  int offB[2][4], offA[2][3];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = 2 * i + (tpp >> 1);
    offB[0][i] = q0 * 128 + 8 * (tpp & 1) + 16 * (c ^ swz(q0));
    offB[1][i] = (q0 + 4) * 128 + 8 * (tpp & 1) + 16 * (c ^ swz(q0 + 4));
  }
#pragma unroll
  for (int sh = 0; sh < 3; ++sh) {
    offA[0][sh] = (q0 + sh) * 128 + 8 * (tpp & 1) + 16 * (ca ^ swz(q0 + sh));
    offA[1][sh] = (q0 + sh + 4) * 128 + 8 * (tpp & 1) + 16 * (ca ^ swz(q0 + sh + 4));
  }

#pragma unroll
  for (int st = 0; st < STAGES - 1; ++st)
    if (st < nks) issue(st, smem + st * BUF);
  // pieces this wave issues per stage (wave-uniform): PPW or PPW - 1
  for (int ks = 0; ks < nks; ++ks) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if (ks + STAGES - 1 < nks) issue(ks + STAGES - 1, smem + ((ks + STAGES - 1) % STAGES) * BUF);
    const char* cur = smem + (ks % STAGES) * BUF;
    const char* db = cur + 3 * XREG + cg * DSUB;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      bf16x8 fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const char* dbi = db + hf * 4096;
        const bf16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(dbi + offB[0][i]));
        const bf16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(dbi + offB[1][i]));
        fb[i] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
      // multi-row segments (W < 64): window pixel p + ds of tap ds = -1 / +1 crosses into the
      // neighbouring image row where w = 0 / W - 1; zero those dY pixels for that tap. This lane
      // holds B rows (pixels) 32 hf + 8 (lane >> 4) + e, e = 0..7 (MFMA 16x16x32 B layout).
      const int pl = 32 * hf + 8 * (lane >> 4);
      const bool mL = MULTIROW && (pl & (a.W - 1)) == 0;      // e = 0 has w = 0
      const bool mR = MULTIROW && ((pl + 8) & (a.W - 1)) == 0;  // e = 7 has w = W - 1
#pragma unroll
      for (int sh = 0; sh < 3; ++sh) {  // ds + 1: window row shift
        bf16x8 fbs[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          fbs[i] = fb[i];
          if (MULTIROW && sh == 0) fbs[i][0] = mL ? (short)0 : fb[i][0];
          if (MULTIROW && sh == 2) fbs[i][7] = mR ? (short)0 : fb[i][7];
        }
#pragma unroll
        for (int r = 0; r < 3; ++r) {  // dr + 1: input row region
          const char* xb = cur + r * XREG + hf * 4096;
          const bf16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(xb + offA[0][sh]));
          const bf16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(xb + offA[1][sh]));
          const bf16x8 fa = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
          const int tap = r * 3 + sh;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[tap][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fbs[i], acc[tap][i], 0, 0, 0);
        }
      }
    }
  }

  // acc[tap][i][r]: cin = cin0 + 16 cf + 4 (lane >> 4) + r, cout = cout0 + 64 cg + 16 i + (lane & 15)
  const auto rs = make_rsrc(a.slab, a.slab_bytes);
  const int cin = cin0 + 16 * cf + 4 * (lane >> 4);
  const int Cin = a.ncols / 9;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = cout0 + 64 * cg + 16 * i + (lane & 15);
    const long rowbase = ((long)split * a.Cout + co) * a.ncols + cin;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const uint32_t off = (uint32_t)(rowbase + t * Cin) * 4u;
      uint4 v;
      v.x = __float_as_uint(acc[t][i][0]); v.y = __float_as_uint(acc[t][i][1]);
      v.z = __float_as_uint(acc[t][i][2]); v.w = __float_as_uint(acc[t][i][3]);
      bstore16(rs, off, v);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Row-ring variant of the halo wgrad for wide rows (W % 64 == 0). K steps walk each 64-pixel
// column (image n, segment wseg) top to bottom: position P = column * H + h. Step P needs input
// rows P - 1, P, P + 1, and rows P - 1 and P were staged by the two previous steps, so a step
// stages ONE new input row region (9 KB) plus its dY tile instead of three regions: half the DMA
// bytes of conv_wgrad_halo_kernel at BN = 64. Input rows live in a 5-slot ring (slot = P % 5), dY
// in a 3-slot ring; two steps stay in flight across the per-step barrier (counted vmcnt). At a
// column's first / last row the dr = -1 / +1 taps are skipped (the neighbouring ring slot holds
// another column's row: that is the zero padding row of this one).
struct WgradRingArgs {
  const u16* x1;
  const u16* x2;
  uint32_t xbytes1, xbytes2;
  int C1, C2, pitch1, pitch2;
  const u16* dy;
  uint32_t dybytes;
  int dypitch;
  float* slab;
  uint32_t slab_bytes;
  int H, W, Cout, ncols;
  int cinTiles, coutTiles, splits, pos_per_split, npos;
  int WS;                           // 64-pixel segments per image row
  uint32_t fh_m, fh_s, fs_m, fs_s;  // fast div by H and by WS
};

template <int BN>
__global__ __launch_bounds__(BN * 4, 2) void conv_wgrad_ring_kernel(const WgradRingArgs a) {
  constexpr int NWV = BN / 16;
  constexpr int XREG = 72 * 128;   // one staged input row region: pixels w0-1 .. w0+70 (66 used)
  constexpr int DSUB = 64 * 128;   // [64 px][64 cout] dY subtile
  constexpr int NX = 5, ND = 3;    // ring slots
  constexpr int DT = (BN / 64) * DSUB;
  constexpr int XPIECES = 9, NPIECES = XPIECES + 8 * (BN / 64);
  constexpr int PPW = (NPIECES + NWV - 1) / NWV;
  constexpr int MINPW = NPIECES / NWV;  // DMAs issued per step by the wave that issues fewest
  __shared__ __attribute__((aligned(16))) char smem[NX * XREG + ND * DT];
  char* const xring = smem;
  char* const dring = smem + NX * XREG;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntiles = a.cinTiles * a.coutTiles;
  const int split = lid / ntiles, tile = lid - split * ntiles;
  const int tc = tile % a.cinTiles, tn = tile / a.cinTiles;
  const int cin0 = tc * 64, cout0 = tn * BN;
  const int p0s = split * a.pos_per_split;
  const int nks = min(a.npos, p0s + a.pos_per_split) - p0s;

  const bool src2 = cin0 >= a.C1;
  const auto rx = src2 ? make_rsrc(a.x2, a.xbytes2) : make_rsrc(a.x1, a.xbytes1);
  const int pitch = src2 ? a.pitch2 : a.pitch1;
  const int ch0 = src2 ? cin0 - a.C1 : cin0;
  const auto rdy = make_rsrc(a.dy, a.dybytes);
  const int rowl = lane >> 3, cpos = lane & 7;

  // position -> (first pixel of the segment, row h); P may be -1 or npos (loads read zeros)
  auto locate = [&](int P, int& m0, int& h, int& w0) {
    const uint32_t up = (uint32_t)max(P, 0);
    const uint32_t col = fdiv2(up, a.fh_m, a.fh_s);
    h = (int)(up - col * (uint32_t)a.H);
    const uint32_t n = fdiv2(col, a.fs_m, a.fs_s);
    const int wseg = (int)(col - n * (uint32_t)a.WS);
    m0 = (((int)n * a.H + h) * a.WS + wseg) * 64;
    w0 = wseg * 64;
    if (P < 0 || P >= a.npos) h = -2;  // no such row: every pixel out of the image
  };
  // piece t of this wave: x-row pieces (when wx) then dY pieces (when wd)
  auto issue = [&](int P, bool wx, bool wd) {
    int m0, h, w0;
    locate(P, m0, h, w0);
#pragma unroll
    for (int t = 0; t < PPW; ++t) {
      const int piece = wave + t * NWV;
      if (piece < XPIECES) {
        if (!wx) continue;
        const int j = piece * 8 + rowl;
        const int g = cpos ^ swz(j);
        const bool ok = (j < 66) & inb(w0 - 1 + j, a.W) & inb(h, a.H);
        const uint32_t off = ok ? (uint32_t)((m0 + j - 1) * pitch + ch0 + g * 8) * 2u : RDP_OOB;
        dma16_async(rx, (lds_void*)(xring + ((P + NX) % NX) * XREG + piece * 1024), off);
      } else if (piece < NPIECES) {
        if (!wd) continue;
        const int d = piece - XPIECES, sub = d >> 3, pj = d & 7;
        const int p = pj * 8 + rowl;
        const int g = cpos ^ swz(p);
        const bool ok = inb(h, a.H);
        const uint32_t off = ok ? (uint32_t)((m0 + p) * a.dypitch + cout0 + sub * 64 + g * 8) * 2u : RDP_OOB;
        dma16_async(rdy, (lds_void*)(dring + (((P - p0s) % ND) * DT) + sub * DSUB + pj * 1024), off);
      }
    }
  };

  f32x4 acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int tg = lane >> 4, tq = (lane >> 2) & 3, tpp = lane & 3;
  const int cf = wave & 3, cg = wave >> 2;
  const int ca = 2 * cf + (tpp >> 1);
  typedef __attribute__((address_space(3))) bf16x4 lds_v4;

  // prologue: rows P0 - 1, P0 (x only), then steps 0 and 1 (row P + 1 and dY P)
  if (nks > 0) {
    issue(p0s - 1, true, false);
    issue(p0s, true, false);
    issue(p0s + 1, true, false);
    issue(p0s, false, true);
    if (nks > 1) { issue(p0s + 2, true, false); issue(p0s + 1, false, true); }
  }
  for (int ks = 0; ks < nks; ++ks) {
    const int P = p0s + ks;
    // step ks's data: everything but the (up to MINPW-per-wave) DMAs of step ks + 1
    if (ks + 1 < nks) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(MINPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if (ks + 2 < nks) { issue(P + 3, true, false); issue(P + 2, false, true); }
    int m0, h, w0;
    locate(P, m0, h, w0);
    const bool top = h == 0, bottom = h == a.H - 1;
    const char* db = dring + ((ks % ND) * DT) + cg * DSUB;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int p0 = 32 * hf + 8 * tg + tq;
      bf16x8 fb[4];
      {
        const int sw0 = swz(p0), sw1 = swz(p0 + 4);
        const int ro0 = p0 * 128 + 8 * (tpp & 1), ro1 = ro0 + 4 * 128;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 2 * i + (tpp >> 1);
          const bf16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(db + ro0 + 16 * (c ^ sw0)));
          const bf16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(db + ro1 + 16 * (c ^ sw1)));
          fb[i] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
        }
      }
#pragma unroll
      for (int sh = 0; sh < 3; ++sh) {
        const int pa = p0 + sh, pb = p0 + sh + 4;
        const int oa = pa * 128 + 8 * (tpp & 1) + 16 * (ca ^ swz(pa));
        const int ob = pb * 128 + 8 * (tpp & 1) + 16 * (ca ^ swz(pb));
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          if ((r == 0 && top) || (r == 2 && bottom)) continue;  // wave-uniform
          const char* xb = xring + ((P + r - 1 + NX) % NX) * XREG;
          const bf16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(xb + oa));
          const bf16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(xb + ob));
          const bf16x8 fa = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
          const int tap = r * 3 + sh;
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[tap][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[i], acc[tap][i], 0, 0, 0);
        }
      }
    }
  }

  const auto rs = make_rsrc(a.slab, a.slab_bytes);
  const int cin = cin0 + 16 * cf + 4 * (lane >> 4);
  const int Cin = a.ncols / 9;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = cout0 + 64 * cg + 16 * i + (lane & 15);
    const long rowbase = ((long)split * a.Cout + co) * a.ncols + cin;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const uint32_t off = (uint32_t)(rowbase + t * Cin) * 4u;
      uint4 v;
      v.x = __float_as_uint(acc[t][i][0]); v.y = __float_as_uint(acc[t][i][1]);
      v.z = __float_as_uint(acc[t][i][2]); v.w = __float_as_uint(acc[t][i][3]);
      bstore16(rs, off, v);
    }
  }
}

// Split-K slab reduction, two levels. A layer's slab is [splits][Cout][ncols_pad] fp32 with up to
// ~500-2000 splits but often only a few 10^4 elements per split (64 x 576 for a 64 -> 64 layer):
// one thread per output walking all splits left ~150 blocks, each latency-bound on a long chain of
// loads (412 us for 75 MB on inc.double_conv.3 at bs64, at the very end of backward). Level 1 sums
// G contiguous groups of splits into the group's first row in place (~1000 blocks, 16-B loads, 4
// independent accumulators); level 2 sums the G group rows into the weight-gradient layout.

// slab rows s0(g) = g * splits / G (g < G) become sum_{s in [s0(g), s0(g+1))} slab[s]
__global__ __launch_bounds__(256) void wgrad_group_sum_kernel(float* __restrict__ slab, long E, int splits, int G) {
  const long e4 = (long)blockIdx.x * 256 + threadIdx.x;  // float4 index within one split row
  if (e4 * 4 >= E) return;
  const int g = blockIdx.y;
  const int s0 = (int)((long)g * splits / G), s1 = (int)((long)(g + 1) * splits / G);
  const float4* p = (const float4*)slab + e4;
  const long st = E >> 2;
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0, a3 = a0;
  int sp = s0;
  for (; sp + 4 <= s1; sp += 4) {
    const float4 v0 = p[(long)sp * st], v1 = p[(long)(sp + 1) * st], v2 = p[(long)(sp + 2) * st],
                 v3 = p[(long)(sp + 3) * st];
    a0.x += v0.x; a0.y += v0.y; a0.z += v0.z; a0.w += v0.w;
    a1.x += v1.x; a1.y += v1.y; a1.z += v1.z; a1.w += v1.w;
    a2.x += v2.x; a2.y += v2.y; a2.z += v2.z; a2.w += v2.w;
    a3.x += v3.x; a3.y += v3.y; a3.z += v3.z; a3.w += v3.w;
  }
  for (; sp < s1; ++sp) {
    const float4 v = p[(long)sp * st];
    a0.x += v.x; a0.y += v.y; a0.z += v.z; a0.w += v.w;
  }
  ((float4*)slab)[(long)s0 * st + e4] = make_float4((a0.x + a1.x) + (a2.x + a3.x), (a0.y + a1.y) + (a2.y + a3.y),
                                                    (a0.z + a1.z) + (a2.z + a3.z), (a0.w + a1.w) + (a2.w + a3.w));
}

// out[cout][tap][cin_real] (+)= sum_g slab[s0(g)][cout][tap*cin_pad + cin]   (s0(g) = g * splits / G)
// V = 4 (cin_real % 4 == 0): each thread owns 4 consecutive outputs, 16-B slab loads / stores (same
// per-element summation order as V = 1; bs 4 step 2.40 -> 2.38 ms)
template <int V>
__global__ void wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out, int splits, int G, int Cout,
                                    int ncols_pad, int taps, int cin_pad, int cin_real, int accumulate) {
  typedef float vf __attribute__((ext_vector_type(V)));
  const long total = (long)Cout * taps * cin_real / V;
  const long stride = (long)Cout * ncols_pad;
  for (long iv = blockIdx.x * (long)blockDim.x + threadIdx.x; iv < total; iv += (long)gridDim.x * blockDim.x) {
    const long idx = iv * V;
    const int cin = idx % cin_real;
    const long t2 = idx / cin_real;
    const int tap = t2 % taps;
    const int co = t2 / taps;
    const long col = (long)tap * cin_pad + cin;
    const float* p = slab + (long)co * ncols_pad + col;
    // 8 independent accumulators: the row loop is latency-bound otherwise
    vf s[8] = {};
    int g = 0;
    for (; g + 8 <= G; g += 8)
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] += *(const vf*)(p + ((long)(g + u) * splits / G) * stride);
    for (; g < G; ++g) s[0] += *(const vf*)(p + ((long)g * splits / G) * stride);
    const vf r = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    *(vf*)(out + idx) = accumulate ? *(const vf*)(out + idx) + r : r;
  }
}

// RDP_ABLATE (profiling only, wrong results): "wgsum" skips the level-1 group sums, "wgred" both levels
static int ablate_flags() {
  static const int f = [] {
    const char* v = getenv("RDP_ABLATE");
    if (!v) return 0;
    return (strstr(v, "wgsum") ? 1 : 0) | (strstr(v, "wgred") ? 2 : 0);
  }();
  return f;
}

extern "C" void rdp_wgrad_reduce(float* slab, float* out, int splits, int Cout, int ncols_pad, int taps, int cin_pad,
                                 int cin_real, int accumulate, hipStream_t s) {
  if (ablate_flags() & 2) return;
  const long E = (long)Cout * ncols_pad;  // multiple of 4 (Cout % 64 == 0)
  const long chunks = (E / 4 + 255) / 256;
  // ~1000 level-1 blocks, at most 32 group rows for level 2; few splits (deep layers) need no level 1
  int G = (int)std::min<long>(std::min<long>(splits, 32), std::max<long>(1, (1024 + chunks - 1) / chunks));
  if (splits <= 8) G = splits;
  if (G < splits && !(ablate_flags() & 1)) hipLaunchKernelGGL(wgrad_group_sum_kernel, dim3((unsigned)chunks, G), dim3(256), 0, s, slab, E, splits, G);
  const long total = (long)Cout * taps * cin_real;
  if (cin_real % 4 == 0 && cin_pad % 4 == 0) {
    const int rb = (int)std::min<long>((total / 4 + 255) / 256, 4096);
    hipLaunchKernelGGL(wgrad_reduce_kernel<4>, dim3(rb), dim3(256), 0, s, slab, out, splits, G, Cout, ncols_pad, taps,
                       cin_pad, cin_real, accumulate);
  } else {
    const int rb = (int)std::min<long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(wgrad_reduce_kernel<1>, dim3(rb), dim3(256), 0, s, slab, out, splits, G, Cout, ncols_pad, taps,
                       cin_pad, cin_real, accumulate);
  }
}

// Which weight-gradient kernel the auto dispatch (variant 0) runs for a 3x3 layer: halo / row-ring where
// whole 64-pixel row segments exist, the generic implicit GEMM for the rest (16^2 maps, packed first
// layer). variant: 0 = auto, 4 = force the generic kernel, 5 = force the halo kernel. (A ping-pong
// 256 x 256 implicit-GEMM wgrad was built and measured 2x slower than the halo kernel: profiles/dead_ends.md.)

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
  // halo-reuse kernel: 3x3, whole 64-pixel row segments
  const bool halo_ok = !packed && taps == 9 && (W % 64 == 0 || (W >= 32 && 64 % W == 0 && (H * W) % 64 == 0)) &&
                       variant != 4;
  if (variant == 5 && !(!packed && taps == 9 && (W % 64 == 0 || (W >= 8 && 64 % W == 0 && (H * W) % 64 == 0))))
    return -1;
  if (halo_ok || variant == 5) {
    WgradHaloArgs h;
    h.x1 = a.x1; h.x2 = a.x2; h.xbytes1 = a.xbytes1; h.xbytes2 = a.xbytes2;
    h.C1 = C1; h.C2 = C2; h.pitch1 = pitch1; h.pitch2 = pitch2;
    h.dy = a.dy; h.dybytes = a.dybytes; h.dypitch = dypitch;
    h.slab = slab; h.H = H; h.W = W; h.Cout = Cout; h.ncols = 9 * a.Cin;
    const int BN = Cout % 128 == 0 ? 128 : 64;
    h.cinTiles = a.Cin / 64; h.coutTiles = Cout / BN;
    const int tiles = h.cinTiles * h.coutTiles;
    h.nseg = a.M / 64;
    // one resident wave of blocks (2/CU at BN = 64, 1/CU at BN = 128), within the slab. (Other grid
    // targets, a minimum segment count per split and the row ring at BN = 128 measured neutral.)
    const int target = BN == 64 ? 512 : 256;
    int sp = std::max(1, (target + tiles - 1) / tiles);
    sp = std::min(sp, std::max(1, h.nseg));
    const long per_split = (long)Cout * h.ncols;
    sp = (int)std::min<long>(sp, slab_elems / per_split);
    if (sp < 1) return -2;
    h.segs_per_split = (h.nseg + sp - 1) / sp;
    h.splits = (h.nseg + h.segs_per_split - 1) / h.segs_per_split;
    if ((long)h.splits * per_split * 4l >= (1l << 31)) return -3;
    h.slab_bytes = (uint32_t)(h.splits * per_split * 4l);
    FastDiv fw = make_fastdiv(W), fh = make_fastdiv(H);
    h.fw_m = fw.m; h.fw_s = fw.s; h.fh_m = fh.m; h.fh_s = fh.s;
    const int nblk = tiles * h.splits;
    if (variant == 0 && W % 64 == 0 && BN == 64) {  // row-ring variant: same split of the positions
      WgradRingArgs g;
      g.x1 = h.x1; g.x2 = h.x2; g.xbytes1 = h.xbytes1; g.xbytes2 = h.xbytes2;
      g.C1 = C1; g.C2 = C2; g.pitch1 = pitch1; g.pitch2 = pitch2;
      g.dy = h.dy; g.dybytes = h.dybytes; g.dypitch = dypitch;
      g.slab = slab; g.slab_bytes = h.slab_bytes; g.H = H; g.W = W; g.Cout = Cout; g.ncols = h.ncols;
      g.cinTiles = h.cinTiles; g.coutTiles = h.coutTiles; g.splits = h.splits;
      g.pos_per_split = h.segs_per_split; g.npos = h.nseg; g.WS = W / 64;
      FastDiv fs = make_fastdiv(W / 64);
      g.fh_m = fh.m; g.fh_s = fh.s; g.fs_m = fs.m; g.fs_s = fs.s;
      hipLaunchKernelGGL((conv_wgrad_ring_kernel<64>), dim3(nblk), dim3(256), 0, s, g);
    } else {
      const bool mr = W < 64;
      if (BN == 128 && mr) hipLaunchKernelGGL((conv_wgrad_halo_kernel<128, true>), dim3(nblk), dim3(512), 0, s, h);
      else if (BN == 128) hipLaunchKernelGGL((conv_wgrad_halo_kernel<128, false>), dim3(nblk), dim3(512), 0, s, h);
      else if (mr) hipLaunchKernelGGL((conv_wgrad_halo_kernel<64, true>), dim3(nblk), dim3(256), 0, s, h);
      else hipLaunchKernelGGL((conv_wgrad_halo_kernel<64, false>), dim3(nblk), dim3(256), 0, s, h);
    }
    rdp_wgrad_reduce(slab, out, h.splits, Cout, h.ncols, 9, a.Cin, a.Cin, accumulate, s);
    return h.splits;
  }
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
  if (packed) hipLaunchKernelGGL((conv_wgrad_kernel<true>), dim3(nblk), dim3(512), 0, s, a);
  else hipLaunchKernelGGL((conv_wgrad_kernel<false>), dim3(nblk), dim3(512), 0, s, a);
  rdp_wgrad_reduce(slab, out, a.splits, Cout, a.ncols_pad, taps, packed ? 8 : a.Cin, packed ? cin_real : a.Cin,
                   accumulate, s);
  return a.splits;
}

// ConvTranspose2d(k=2, s=2) weight gradient straight from its output gradient du [N][H2][W2][C] (the
// window 2h x 2w at (oy, ox)) and its input x [N][h][w][Cin]: out[ci][(sub, c)] (+)= sum_px
// x[px][ci] du[sub-pixel sub of px][c] -- the generic kernel's role-swapped GEMM (columns = the 4
// sub-pixels x C, "couts" = Cin) reading du at the sub-pixels instead of an unshuffled copy.
// Returns the split count, or < 0 if the shape does not fit.
extern "C" int rdp_conv_wgrad_upT(const void* du, long dubytes, int C, int dupitch, int H2, int W2, int oy, int ox,
                                  const void* x, long xbytes, int Cin, int xpitch, int N, int h, int w, float* slab,
                                  long slab_elems, float* out, int accumulate, int splits, hipStream_t s) {
  if (C % 64 || Cin % 64 || oy < 0 || ox < 0 || 2 * h + oy > H2 || 2 * w + ox > W2) return -1;
  if (dubytes >= (1l << 31) || xbytes >= (1l << 31)) return -1;
  WgradArgs a;
  a.x1 = (const u16*)du; a.x2 = nullptr; a.xbytes1 = (uint32_t)dubytes; a.xbytes2 = 0;
  a.C1 = C; a.C2 = 0; a.pitch1 = dupitch; a.pitch2 = dupitch;
  a.dy = (const u16*)x; a.dybytes = (uint32_t)xbytes; a.dypitch = xpitch;
  a.slab = slab; a.H = h; a.W = w; a.M = N * h * w; a.Cout = Cin;
  a.taps = 4; a.packed = 0; a.Cin = C; a.ncols = 4 * C;
  a.uH2 = H2; a.uW2 = W2; a.uoy = oy; a.uox = ox;
  a.colTiles = (a.ncols + 255) / 256;
  a.ncols_pad = a.colTiles * 256;
  a.coutTiles = Cin / 64;
  if (splits < 1) splits = 1;
  int pps = (a.M + splits - 1) / splits;
  pps = (pps + 63) / 64 * 64;
  a.pix_per_split = pps;
  a.splits = (a.M + pps - 1) / pps;
  if ((long)a.splits * a.Cout * a.ncols_pad > slab_elems) return -2;
  if ((long)a.splits * a.Cout * a.ncols_pad * 4l >= (1l << 31)) return -3;
  FastDiv fw = make_fastdiv(w), fh = make_fastdiv(h);
  a.fw_m = fw.m; a.fw_s = fw.s; a.fh_m = fh.m; a.fh_s = fh.s;
  const int nblk = a.colTiles * a.coutTiles * a.splits;
  hipLaunchKernelGGL((conv_wgrad_kernel<false, true>), dim3(nblk), dim3(512), 0, s, a);
  rdp_wgrad_reduce(slab, out, a.splits, Cin, a.ncols_pad, 4, C, C, accumulate, s);
  return a.splits;
}

// ---------------------------------------------------------------------------------------------
// First layer (inc.double_conv.0, 3 -> 64, reference /root/reference/pkg/segmentation_model.py:31):
// BN-backward apply + ReLU mask fused into the weight gradient. The first conv has no input
// gradient, so its pre-BN gradient dz = A * relu_mask(y) * da + B * y + K (the bn_relu_bwd_apply
// formula, norm_act.hip) is consumed ONLY by this wgrad: computing it here, in registers, and staging
// it straight into the LDS dY tile drops the 537 MB dz write + re-read of a bs-64 step (the separate
// apply pass plus the packed wgrad's dY stream) at the end of backward, where it sits on the
// critical path.
//
// Per 64-pixel K step a block stages: x taps 0..7 (8 channels each, channel 3..7 the stored zero pad)
// and tap 8 by LDS-DMA (the packed layout of conv_wgrad_kernel<PACKED>), and dz [64 px][64 couts]
// computed from da / y by every thread (channel group tc = tid & 7 fixed per thread, so the 40
// BN coefficients stay in registers; swizzle applied on the LDS write address). Only the 80 valid
// (tap, channel) columns are multiplied (5 MFMA column fragments instead of the packed kernel's 16).
// Wave w owns couts 16w .. 16w + 15. The dz loads of step k + 1 are issued before step k's MFMAs and
// written to the other LDS buffer after them (one barrier per step). Slab [splits][64][80] fp32,
// reduced by the shared two-level wgrad reduction.
struct FirstWgradArgs {
  const u16* x;
  uint32_t xbytes;
  int xpitch;
  const u16* da;
  uint32_t dabytes;
  int dapitch;
  const u16* y;
  uint32_t ybytes;
  int ypitch;
  const float* coef;   // [mean | invstd | scale | shift] x 64
  const float* coef2;  // [A | B | K] x 64 (bn_bwd_finalize)
  float* slab;
  uint32_t slab_bytes;
  int H, W, M, pix_per_split;
  uint32_t fw_m, fw_s, fh_m, fh_s;
};
constexpr int FWG_NCOLS = 80;

RDP_DEV void fw_unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__global__ __launch_bounds__(256, 2) void wgrad_first_bn_kernel(const FirstWgradArgs a) {
  constexpr int SUB = 64 * 128;  // [64 px][64 bf16]
  constexpr int BUF = 3 * SUB;   // x taps 0..7 | x tap 8 | dz
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int split = (int)xcd_remap(blockIdx.x, gridDim.x);
  const int pbeg = split * a.pix_per_split;
  const int nks = max(0, min(a.M, pbeg + a.pix_per_split) - pbeg) / 64;  // host: multiples of 64
  const auto rx = make_rsrc(a.x, a.xbytes);
  const auto rda = make_rsrc(a.da, a.dabytes);
  const auto ry = make_rsrc(a.y, a.ybytes);

  // dz producer role: channel group tc (fixed), pixel rows tr0 and tr0 + 32 of each K step
  const int tc = threadIdx.x & 7, tr0 = threadIdx.x >> 3;
  float ss[8], hh[8], cA[8], cB[8], cK[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = 8 * tc + k;
    ss[k] = a.coef[128 + c]; hh[k] = a.coef[192 + c];
    cA[k] = a.coef2[c]; cB[k] = a.coef2[64 + c]; cK[k] = a.coef2[128 + c];
  }
  uint4 vd[2], vy[2];
  auto load_dz = [&](int ks) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int m = pbeg + ks * 64 + tr0 + 32 * u;
      vd[u] = bload16(rda, (uint32_t)(m * a.dapitch + 8 * tc) * 2u);
      vy[u] = bload16(ry, (uint32_t)(m * a.ypitch + 8 * tc) * 2u);
    }
  };
  auto store_dz = [&](char* buf) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = tr0 + 32 * u;
      float fd[8], fy[8];
      fw_unpack8(vd[u], fd);
      fw_unpack8(vy[u], fy);
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 8; k += 2) {
        const float g0 = fmaf(fy[k], ss[k], hh[k]) > 0.f ? fd[k] : 0.f;
        const float g1 = fmaf(fy[k + 1], ss[k + 1], hh[k + 1]) > 0.f ? fd[k + 1] : 0.f;
        o[k / 2] = pack2bf(fmaf(cA[k], g0, fmaf(cB[k], fy[k], cK[k])),
                           fmaf(cA[k + 1], g1, fmaf(cB[k + 1], fy[k + 1], cK[k + 1])));
      }
      *(uint4*)(buf + 2 * SUB + p * 128 + 16 * (tc ^ swz(p))) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  };
  const int rowl = lane >> 3, cpos = lane & 7;
  // x: 16 DMA pieces (2 subtiles x 8 pieces of 8 pixel rows), 4 per wave
  auto issue_x = [&](int ks, char* buf) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int s = wave * 4 + t, sub = s >> 3, pj = s & 7;
      const int p = pj * 8 + rowl;
      const int g = cpos ^ swz(p);
      const int m = pbeg + ks * 64 + p;
      const uint32_t q = fdiv2((uint32_t)m, a.fw_m, a.fw_s);
      const int w = m - (int)q * a.W;
      const int h = (int)q - (int)fdiv2(q, a.fh_m, a.fh_s) * a.H;
      const int tap = sub * 8 + g;
      const int dr = tap / 3 - 1, ds = tap % 3 - 1;
      const bool ok = (tap < 9) & inb(h + dr, a.H) & inb(w + ds, a.W);
      const uint32_t off = ok ? (uint32_t)((m + dr * a.W + ds) * a.xpitch) * 2u : RDP_OOB;
      dma16_async(rx, (lds_void*)(buf + sub * SUB + pj * 1024), off);
    }
  };

  f32x4 acc[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int tg = lane >> 4, tq = (lane >> 2) & 3, tpp = lane & 3;
  typedef __attribute__((address_space(3))) bf16x4 lds_v4;

  if (nks > 0) {
    load_dz(0);
    issue_x(0, smem);
    store_dz(smem);
  }
  for (int ks = 0; ks < nks; ++ks) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    raw_barrier();
    const char* cur = smem + (ks & 1) * BUF;
    char* nxt = smem + ((ks + 1) & 1) * BUF;
    const bool more = ks + 1 < nks;
    if (more) {
      load_dz(ks + 1);
      issue_x(ks + 1, nxt);
    }
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int p0 = 32 * hf + 8 * tg + tq;
      const int sw0 = swz(p0), sw1 = swz(p0 + 4);
      const int ro0 = p0 * 128 + 8 * (tpp & 1), ro1 = ro0 + 4 * 128;
      auto frag = [&](const char* base, int i) {
        const int c = 2 * i + (tpp >> 1);
        const bf16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(base + ro0 + 16 * (c ^ sw0)));
        const bf16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(base + ro1 + 16 * (c ^ sw1)));
        return __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
      };
      const bf16x8 fb = frag(cur + 2 * SUB, wave);
      bf16x8 fa[5];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag(cur, i);
      fa[4] = frag(cur + SUB, 0);
#pragma unroll
      for (int i = 0; i < 5; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb, acc[i], 0, 0, 0);
    }
    if (more) store_dz(nxt);
  }

  // acc[i][r]: col = 16 i + 4 (lane >> 4) + r, cout = 16 wave + (lane & 15)
  const auto rs = make_rsrc(a.slab, a.slab_bytes);
  const int co = 16 * wave + (lane & 15);
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int col = 16 * i + 4 * (lane >> 4);
    const uint32_t off = (uint32_t)(((long)split * 64 + co) * FWG_NCOLS + col) * 4u;
    uint4 v;
    v.x = __float_as_uint(acc[i][0]); v.y = __float_as_uint(acc[i][1]);
    v.z = __float_as_uint(acc[i][2]); v.w = __float_as_uint(acc[i][3]);
    bstore16(rs, off, v);
  }
}

// Returns the number of splits, or < 0 (nothing launched) when the shape does not fit this kernel.
extern "C" int rdp_wgrad_first_bn(const void* x, long xbytes, int xpitch, const void* da, long dabytes, int dapitch,
                                  const void* y, long ybytes, int ypitch, const float* coef, const float* coef2,
                                  float* slab, long slab_elems, float* out, int accumulate, int N, int H, int W,
                                  int cin_real, int splits, hipStream_t s) {
  const long M = (long)N * H * W;
  if (M % 64 || cin_real > 8 || cin_real < 1) return -1;
  if (xbytes >= (1l << 31) || dabytes >= (1l << 31) || ybytes >= (1l << 31)) return -1;
  if (xpitch % 8 || dapitch % 8 || ypitch % 8) return -1;
  splits = (int)std::max(1L, std::min<long>(splits, M / 64));
  long pps = (M + splits - 1) / splits;
  pps = (pps + 63) / 64 * 64;
  splits = (int)((M + pps - 1) / pps);
  const long per_split = 64l * FWG_NCOLS;
  if ((long)splits * per_split > slab_elems) return -2;
  if ((long)splits * per_split * 4l >= (1l << 31)) return -3;
  FirstWgradArgs a;
  a.x = (const u16*)x; a.xbytes = (uint32_t)xbytes; a.xpitch = xpitch;
  a.da = (const u16*)da; a.dabytes = (uint32_t)dabytes; a.dapitch = dapitch;
  a.y = (const u16*)y; a.ybytes = (uint32_t)ybytes; a.ypitch = ypitch;
  a.coef = coef; a.coef2 = coef2;
  a.slab = slab; a.slab_bytes = (uint32_t)(splits * per_split * 4l);
  a.H = H; a.W = W; a.M = (int)M; a.pix_per_split = (int)pps;
  FastDiv fw = make_fastdiv(W), fh = make_fastdiv(H);
  a.fw_m = fw.m; a.fw_s = fw.s; a.fh_m = fh.m; a.fh_s = fh.s;
  hipLaunchKernelGGL(wgrad_first_bn_kernel, dim3(splits), dim3(256), 0, s, a);
  rdp_wgrad_reduce(slab, out, splits, 64, FWG_NCOLS, 9, 8, cin_real, accumulate, s);
  return splits;
}

// Slab size (elements) for the generic kernel's `splits` pixel splits. The halo / row-ring kernels choose
// their own split count, capped by the slab they are given: the training step shares one slab of the
// largest generic size, which caps the deep layers' halo wgrads at 4-15 splits (~120 blocks). That is
// deliberate: sized for a full wave of halo blocks (rdp_conv_wgrad_halo_slab_elems) the wgrads run ~1.8x
// faster alone but the step got slower -- bs 64 3,120-3,131 vs 3,160-3,181 img/s, bs 4 1,405-1,409 vs
// 1,591 (same box, 2 rounds): the side-stream wgrads then take every CU from the main stream's convs.
extern "C" long rdp_conv_wgrad_slab_elems(int N, int H, int W, int Cin, int Cout, int taps, int packed, int splits) {
  const int ncols = packed ? 72 : taps * Cin;
  const int ncols_pad = (ncols + 255) / 256 * 256;
  const long M = (long)N * H * W;
  long pps = (M + splits - 1) / splits;
  pps = (pps + 63) / 64 * 64;
  const long sp = (M + pps - 1) / pps;
  return sp * Cout * ncols_pad;
}

// Slab the halo / row-ring wgrad needs for one resident wave of blocks (its own split choice
// unconstrained); 0 where the dispatch does not pick those kernels. (conv_microbench.py sizes with it.)
extern "C" long rdp_conv_wgrad_halo_slab_elems(int N, int H, int W, int Cin, int Cout) {
  const long M = (long)N * H * W;
  const bool halo = Cin % 64 == 0 && Cout % 64 == 0 && (W % 64 == 0 || (W >= 32 && 64 % W == 0 && (H * W) % 64 == 0));
  if (!halo) return 0;
  const int BN = Cout % 128 == 0 ? 128 : 64;
  const long tiles = (long)(Cin / 64) * (Cout / BN);
  const long target = BN == 64 ? 512 : 256;
  long hsp = std::max<long>(1, (target + tiles - 1) / tiles);
  hsp = std::min<long>(hsp, std::max<long>(1, M / 64));
  return hsp * Cout * 9L * Cin;
}
